# bench.py headline at N=1, plain vs the one-rank RCCL path (WCE_FORCE_DIST=1), alternated
set -o pipefail
# EXTRA: more bench flags (e.g. EXTRA="--prewarm-s 2")
O=gpurun_out/forcedist_ab.txt; : > $O
for i in 1 2; do
  timeout -k 10 120 python3 bench.py --no-extras --no-cpu-baseline $EXTRA 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('plain', d['ms_per_step'], d['timed_region_ms'])" >> $O || exit $?
  WCE_FORCE_DIST=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=2953$i RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 timeout -k 10 120 python3 bench.py --no-extras --no-cpu-baseline $EXTRA 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('fd   ', d['ms_per_step'], d['timed_region_ms'])" >> $O || exit $?
done
