/*
 * wce_compat.h -- the reference's five estimator entry points, with the exact
 * signatures of main.c:4-8, implemented by libwce.so on the GPU.
 *
 * One frame, host memory, long double _Complex arrays of 53 (SAMPUTIL) as in
 * the reference.  Values are converted to fp64, run through the batched
 * engine (wce.h) with B = 1 on the default device, and converted back.
 * A maintainer replaces the bodies in main.c with these.
 *
 * PS_MMSE computes the REF-repaired result (wce.h WCE_MMSE_REF): the
 * reference's own pipeline returns NaN on every subcarrier because its
 * cofactor inverse of Ryy divides 0/0 (utils.c:557) -- see DESIGN.md.
 * Errors cannot be returned through these void signatures; they are
 * reported by wce_compat_last_status().
 */
#ifndef WCE_COMPAT_H
#define WCE_COMPAT_H

#ifdef __cplusplus
extern "C" {
#endif

/* main.c:4 */
void WiFi_channel_estimation_LT_LS(long double _Complex tx_pre[], long double _Complex rx_pre[],
                                   long double _Complex H_EST[]);
/* main.c:5 */
void WiFi_channel_estimation_PS_Linear(long double _Complex tx_symbols[],
                                       long double _Complex rx_symbols[],
                                       long double _Complex H_EST[]);
/* main.c:6 */
void WiFi_channel_estimation_PS_Cubic(long double _Complex tx_symbols[],
                                      long double _Complex rx_symbols[],
                                      long double _Complex H_EST[]);
/* main.c:7 */
void WiFi_channel_estimation_PS_Sinc(long double _Complex tx_symbols[],
                                     long double _Complex rx_symbols[],
                                     long double _Complex H_EST[]);
/* main.c:8 */
void WiFi_channel_estimation_PS_MMSE(long double _Complex tx_symbols[],
                                     long double _Complex rx_symbols[],
                                     long double _Complex **F, double ow2,
                                     long double _Complex H_EST_LS[],
                                     long double _Complex H_EST[]);

/* status of the last compat call (0 = ok, wce.h error codes otherwise) */
int wce_compat_last_status(void);

#ifdef __cplusplus
}
#endif
#endif /* WCE_COMPAT_H */
