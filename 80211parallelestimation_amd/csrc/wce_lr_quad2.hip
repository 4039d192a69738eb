// wce_lr_quad2.hip -- WCE_MMSE_COV at ranks 17..32 of a power-delay profile
// with taps 0..r-1 (round 6): mmse_lr_quad2_kernel, its own translation unit
// (its unrolled 20..32-row Cholesky compiles in parallel with wce_kernels.hip).
#include "wce_internal.h"
#include "wce_device.h"

namespace wce {

// ---------------------------------------------------------------------
// Ranks 17..32 of a power-delay profile with taps 0..R-1 (State::taps_contig,
// round 6): the quad kernel's 16-lane Toeplitz form with TWO rows per lane.
// Lane i of a 16-lane DPP row holds row i of the R x R system in Ar (columns
// 0..15 only: row i < 16 needs j <= i) and row i + 16 in Br (lanes i < R - 16).
// Every broadcast stays inside the DPP row (row_newbcast:n from lane n of the
// set that holds the source row), so the 53-row block-cyclic machinery of the
// wave kernel (0.33 ms per 65,536 frames at rank 24, 20% of FP64 peak) is not
// needed:
//   Gram     Q(i), Q(i + 16) and beta_i, beta_{i+16}: two DFTs per lane over
//            the frame's |x|^2 and conj(x) rx, E[k d mod 53] from LDS by the
//            exact index recurrence (as the quad kernel)
//   Cholesky pivot C < 16 updates Ar[j] (j < 16) and Br[j]; C >= 16 Br only
//   z = L^-1 beta column by column, z_c as the DPP64 operand of the FMAs
//            (round 6); t = L^-H z by 16-lane DPP sums
//   complex x: the quad kernel's correction term; H_k = sum_j s_j t_j E[k j]
//            over the pairs (k, 53 - k), the DFTs' broadcasts fused into DPP64 FMAs
// Same algebra as mmse_lr_quad_kernel / mmse_lr_kernel, summed in another
// order (~1e-15).
// ---------------------------------------------------------------------
// acc -= l conj(L[j][C]) with L[j][C] from lane (j mod 16) of column register R
template <bool FD>
__device__ __forceinline__ void chol_upd(int n, double2 &acc, double2 l, double2 R)
{
    if constexpr (FD) cmsub_dpp_n(n, acc, l, R);
    else cmsub_conj(acc, l, row_bcast_n(R, n));
}

template <int R, int C, bool FD>
__device__ __forceinline__ void lrq2_chol(double2 (&Ar)[16], double2 (&Br)[R], double &lda, double &ldb, int i)
{
    if constexpr (C < R) {
        if constexpr (C < 16) {
            const double rs = rsq_nr(row_bcast<C>(Ar[C]).x);   // pivot (C, C) from lane C's row
            Ar[C] = cscale(Ar[C], rs);                        // L[i][C], L[i + 16][C]
            Br[C] = cscale(Br[C], rs);
            lda = i == C ? rs : lda;
            if constexpr (FD) dpp_ready(Ar[C], Br[C]);
#pragma unroll
            for (int j = C + 1; j < 16; ++j) {                // rows i >= j of both sets
                chol_upd<FD>(j, Ar[j], Ar[C], Ar[C]);
                chol_upd<FD>(j, Br[j], Br[C], Ar[C]);
            }
#pragma unroll
            for (int j = 16; j < R; ++j)                      // rows i + 16 >= j only
                chol_upd<FD>(j - 16, Br[j], Br[C], Br[C]);
        } else {
            const double rs = rsq_nr(row_bcast<C - 16>(Br[C]).x);
            Br[C] = cscale(Br[C], rs);
            ldb = i == C - 16 ? rs : ldb;
            if constexpr (FD) dpp_ready(Br[C], Br[C]);
#pragma unroll
            for (int j = C + 1; j < R; ++j) chol_upd<FD>(j - 16, Br[j], Br[C], Br[C]);
        }
        lrq2_chol<R, C + 1, FD>(Ar, Br, lda, ldb, i);
    }
}

// One unit's LDS: the Gram's tables.  The unit pitch (216 slots of 16 B, 8 mod
// 16) puts two units' same-index reads (the pair tables' broadcasts,
// Q(|r - j|)) in one ds_read_b128 lane group on different banks.
struct Lrq2Tabs {
    double2 Q[33];                    // Q(0..31)
    double2 V[56];                    // conj(x_k) rx_k ...
    double W[56];                     // ... and |x_k|^2
    double2 PA[33], PB[33], RP[33];   // the pair tables (k = 1..26)
};
static_assert(sizeof(Lrq2Tabs) / 16 % 16 == 8, "unit pitch 8 mod 16 slots");

// the forward substitution's column C (compile-time, so that every DPP lane
// select is an immediate and nothing is left to the unroller): z_C = y_C / L_CC
// from lane C (mod 16), conjugated for cmsub_dpp, then y_r -= L[r][C] z_C
template <int R, int C>
__device__ __forceinline__ void lrq2_fwd(const double2 (&Ar)[16], const double2 (&Br)[R], double2 &ya, double2 &yb,
                                         double lda, double ldb)
{
    if constexpr (C < R) {
        if constexpr (C < 16) {
            double2 w = make_double2(ya.x * lda, -(ya.y * lda));
            dpp_ready(w);
            cmsub_dpp<C>(ya, Ar[C], w);
            cmsub_dpp<C>(yb, Br[C], w);
        } else {
            double2 w = make_double2(yb.x * ldb, -(yb.y * ldb));
            dpp_ready(w);
            cmsub_dpp<C - 16>(yb, Br[C], w);
        }
        lrq2_fwd<R, C + 1>(Ar, Br, ya, yb, lda, ldb);
    }
}

template <int R, bool FD = true, int MINW = 2>
__global__ __launch_bounds__(256, MINW) void mmse_lr_quad2_kernel(const State *__restrict__ st, SolveArgs a)
{
    static_assert(R > 16 && R <= 32, "two rows per lane");
    constexpr int R2 = R - 16;
    const int i = threadIdx.x & 15;                   // rows i and i + 16 of the system
    const int rw = (threadIdx.x >> 4) & 15;           // the unit's 16-lane row in the workgroup
    const int64_t units = a.split ? a.n * a.nblk : a.n;
    const int64_t g = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
    __shared__ double2 sE[64];
    __shared__ Lrq2Tabs sU[16];   // the workgroup's 16 units
    Lrq2Tabs &T = sU[rw];
    if (threadIdx.x < 64) sE[threadIdx.x] = ld2(st->dft, threadIdx.x);
    __syncthreads();
    if (g >= units || (a.skip && a.skip[g])) return;   // whole 16-lane rows
    const int64_t f = a.split ? g / a.nblk : g;
    const int b = a.split ? (int)(g - f * a.nblk) : 0;
    const int64_t base = f * a.fs + (int64_t)(a.blk + b) * a.bs;
    const double ac = st->acoef, bc = st->bcoef;
    const uint64_t xm = st->xmask;
    const bool rowb = i < R2;
    bool cplx = false;
#pragma unroll
    for (int m = 0; m < 4; ++m) {   // the frame through LDS: 256 B per row and instruction
        const int k = i + 16 * m;
        if (k < NSC) {
            double2 x = ld2(a.tx, base + k);
            const double2 r = ld2(a.rx, base + k);
            if (!((xm >> k) & 1ull)) x = make_double2(0.0, 0.0);
            cplx |= x.y != 0.0;
            T.W[k] = fma(x.x, x.x, x.y * x.y);
            T.V[k] = make_double2(fma(x.x, r.x, x.y * r.y), fma(x.x, r.y, -x.y * r.x));   // conj(x) rx
        }
    }
    wave_lds_sync();
    // pair tables over (k, 53 - k), k = 1..26: conj(E[(53 - k) d]) = E[k d], so
    //   p_k conj(E) + p_{53-k} E = (p_k + p_{53-k}) Re E - i (p_k - p_{53-k}) Im E
    //   v_k conj(E) + v_{53-k} E = (v_k + v_{53-k}) Re E - i (v_k - v_{53-k}) Im E
    // -- one gather and half the FMAs per pair (the wave kernel's dft_pairs)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int k = i + 1 + 16 * h;
        if (k <= NSC / 2) {
            const double2 u = T.V[k], w = T.V[NSC - k];
            const double pu = T.W[k], pw = T.W[NSC - k];
            T.PA[k] = cadd(u, w);
            T.PB[k] = csub(u, w);
            T.RP[k] = make_double2(pu + pw, pu - pw);
        }
    }
    wave_lds_sync();
    // Q(d) = sum_k p_k conj(E[k d]) and sum_k v_k conj(E[k d]) at d = i and d = i + 16
    double2 qa = make_double2(T.W[0], 0.0), qb = qa, ba = T.V[0], bb = ba;   // the k = 0 terms
    {
        const uint32_t sa = 16u * (uint32_t)i, swa = sa - 16u * NSC;
        const uint32_t sb = 16u * (uint32_t)(i + 16), swb = sb - 16u * NSC;
        uint32_t oa = sa, ob = sb;   // k = 1
#pragma unroll 2
        for (int k = 1; k <= NSC / 2; ++k) {
            const double2 ea = ld_e(sE, oa), eb = ld_e(sE, ob), pa = T.PA[k], pb = T.PB[k], pp = T.RP[k];
            qa.x = fma(pp.x, ea.x, qa.x);
            qa.y = fma(-pp.y, ea.y, qa.y);
            qb.x = fma(pp.x, eb.x, qb.x);
            qb.y = fma(-pp.y, eb.y, qb.y);
            ba.x = fma(pa.x, ea.x, fma(pb.y, ea.y, ba.x));
            ba.y = fma(pa.y, ea.x, fma(-pb.x, ea.y, ba.y));
            bb.x = fma(pa.x, eb.x, fma(pb.y, eb.y, bb.x));
            bb.y = fma(pa.y, eb.x, fma(-pb.x, eb.y, bb.y));
            oa = dft_step(oa, sa, swa);
            ob = dft_step(ob, sb, swb);
        }
    }
    const double sia = st->col_s[i], sib = rowb ? st->col_s[i + 16] : 0.0;
    T.Q[i] = qa;
    T.Q[i + 16] = qb;
    wave_lds_sync();
    double2 Ar[16], Br[R];   // a s_r s_j Q(r - j) + b [r == j]  (Q(-d) = conj(Q(d)))
    // one LDS read per element: |r - j| indexes Q, the sign picks the conjugate
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int d = i - j;
        double2 qd = T.Q[d >= 0 ? d : -d];
        qd.y = d >= 0 ? qd.y : -qd.y;
        Ar[j] = cscale(qd, ac * sia * st->col_s[j]);
        Ar[j].x += i == j ? bc : 0.0;
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const int d = i + 16 - j;
        double2 qd = T.Q[d >= 0 ? d : -d];
        qd.y = d >= 0 ? qd.y : -qd.y;
        Br[j] = cscale(qd, ac * sib * st->col_s[j]);   // zero on lanes without a second row
        Br[j].x += (rowb && i + 16 == j) ? bc : 0.0;
    }
    double lda = 1.0, ldb = 1.0;
    lrq2_chol<R, 0, FD>(Ar, Br, lda, ldb, i);
    // z = L^-1 beta (beta_r = s_r sum_k v_k conj(E[k r])): lane i keeps
    // y_i = beta_i - sum_{c < i} L[i][c] z_c and y_{i+16}; z_c = y_c / L_cc from
    // lane c (mod 16) as the DPP64 row_newbcast operand (conj(z_c) in w:
    // cmsub_dpp subtracts l conj(R)).  L's entries on and above the diagonal
    // are zeroed first, so that no lane needs a select here or in the
    // back-substitution (round 6, as mmse_lr_quad_kernel).
#pragma unroll
    for (int c = 0; c < 16; ++c) keep_where_mask(rows16_upto(c), true, Ar[c], make_double2(0.0, 0.0));
#pragma unroll
    for (int c = 16; c < R; ++c) keep_where_mask(rows16_upto(c - 16), true, Br[c], make_double2(0.0, 0.0));
    double2 ya = cscale(ba, sia), yb = cscale(bb, sib);
    lrq2_fwd<R, 0>(Ar, Br, ya, yb, lda, ldb);
    const double2 za = cscale(ya, lda), zb = cscale(yb, ldb);
    // t = L^-H z: t_c = (z_c - sum_{m > c} conj(L[m][c]) t_m) / L_cc, the sum
    // over both sets of the row (lanes whose rows are not below c hold a zero
    // or a t still zero)
    double2 ta = make_double2(0.0, 0.0), tb = ta;
#pragma unroll
    for (int c = R - 1; c >= 0; --c) {
        double2 term = cmul(cconj(Br[c]), tb);
        if (c < 16) term = cadd(term, cmul(cconj(Ar[c < 16 ? c : 0]), ta));
        const double2 sum = row16_sum(term);
        if (c < 16) {
            if (i == c) ta = cscale(csub(za, sum), lda);
        } else if (i == c - 16) {
            tb = cscale(csub(zb, sum), ldb);
        }
    }
    double *W = a.w + 2 * g * a.ws;
    if (__ballot(cplx) != 0) {   // complex symbols, in the tap domain (round 6): see lrq_cplx_taps
        double2 ca = cscale(ta, sia), cb = cscale(tb, sib);
        lrq_cplx_taps<R>(xm, a.tx, a.rx, base, sE, T.V, ca, cb, i, ac, bc);
        ta = cadd(ta, cscale(ca, sia));
        tb = cadd(tb, cscale(cb, sib));
    }
    // H_k = sum_j s_j t_j E[k j] over the pairs (k, 53 - k): with c_j = s_j t_j,
    // A = sum_j c_j Re E[k j], B = sum_j c_j Im E[k j], H_k = A + i B and
    // H_{53-k} = A - i B.  Lane i: k = i + 1 and i + 17 (<= 26); H_0 = sum_j c_j
    // over the row.  c_j reaches the FMAs as their DPP64 row_newbcast operand.
    const double2 ca = cscale(ta, sia), cb = cscale(tb, sib);
    const double2 h0 = row16_sum(cadd(ca, cb));
    const int k1 = i + 1, k2 = i + 17;
    const bool two = k2 <= NSC / 2;
    const uint32_t s1 = 16u * (uint32_t)k1, w1 = s1 - 16u * NSC;
    const uint32_t s2 = 16u * (uint32_t)(two ? k2 : k1), w2 = s2 - 16u * NSC;
    uint32_t o1 = 0, o2 = 0;
    double2 A1 = make_double2(0.0, 0.0), B1 = A1, A2 = A1, B2 = A1;
    double2 cav = ca, cbv = cb;
    dpp_ready(cav, cbv);
    lrq2_readout<R, 0>(sE, cav, cbv, o1, o2, s1, w1, s2, w2, A1, B1, A2, B2);
    if (i == 0) st2(W, 0, h0);
    st2(W, k1, make_double2(A1.x - B1.y, A1.y + B1.x));
    st2(W, NSC - k1, make_double2(A1.x + B1.y, A1.y - B1.x));
    if (two) {
        st2(W, k2, make_double2(A2.x - B2.y, A2.y + B2.x));
        st2(W, NSC - k2, make_double2(A2.x + B2.y, A2.y - B2.x));
    }
}

int launch_lr_quad2(const State *st, int rank, const SolveArgs &a, void *stream, int form)
{
    // instantiated at 20, 24, 28, 32 rows: a rank r below runs the next size
    // up with rows r.. as b I (col_s = 0 past the rank: no coupling, t = 0
    // there), bitwise the same arithmetic on the live rows.  Built for 2 waves
    // per SIMD (216 / 242 / 256 / 256 VGPRs at 20 / 24 / 28 / 32; 28 and 32
    // spill 28 / 116 B per lane since round 6's forward substitution, 192 /
    // 236 B before): 65,536 frames at rank 24 154.5 us against 225.6 us left at
    // 1 wave per SIMD (20 / 28 / 32: 130 / 241 / 278 against 133 / 255 / 278;
    // profiles/r06_ab_lowrank.txt); after the solve change 28 / 32: 161 / 198
    // against 232 / 256 us (profiles/r06_ab_lowrank_minw.txt).
    // form (A/B): 0 the product, 1 the Cholesky's broadcasts as separate movs
    // (rank 21..24 only), 2 every size at 1 wave per SIMD (no spills)
    if (rank <= 16 || rank > 32) return WCE_EINVAL;
    const int64_t units = a.split ? a.n * a.nblk : a.n;
    const dim3 gq((unsigned)((units + 15) / 16)), bq(256);
    hipStream_t s = (hipStream_t)stream;
    if (form == 1 && rank > 20 && rank <= 24)
        hipLaunchKernelGGL((mmse_lr_quad2_kernel<24, false, 2>), gq, bq, 0, s, st, a);
    else if (form == 2) {
        if (rank <= 20) hipLaunchKernelGGL((mmse_lr_quad2_kernel<20, true, 1>), gq, bq, 0, s, st, a);
        else if (rank <= 24) hipLaunchKernelGGL((mmse_lr_quad2_kernel<24, true, 1>), gq, bq, 0, s, st, a);
        else if (rank <= 28) hipLaunchKernelGGL((mmse_lr_quad2_kernel<28, true, 1>), gq, bq, 0, s, st, a);
        else hipLaunchKernelGGL((mmse_lr_quad2_kernel<32, true, 1>), gq, bq, 0, s, st, a);
    } else if (rank <= 20) hipLaunchKernelGGL((mmse_lr_quad2_kernel<20>), gq, bq, 0, s, st, a);
    else if (rank <= 24) hipLaunchKernelGGL((mmse_lr_quad2_kernel<24>), gq, bq, 0, s, st, a);
    else if (rank <= 28) hipLaunchKernelGGL((mmse_lr_quad2_kernel<28>), gq, bq, 0, s, st, a);
    else hipLaunchKernelGGL((mmse_lr_quad2_kernel<32>), gq, bq, 0, s, st, a);
    return hipGetLastError() == hipSuccess ? WCE_OK : WCE_EHIP;
}

}  // namespace wce
