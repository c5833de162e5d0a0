#!/bin/bash
# Round 6, pass e: what the post-loop time of the path-6 waves is (timelines, A/B knobs):
# no statistics atomics, no x̄ epilogue, both; one lane without the folded step.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6e
mkdir -p $O
export TMPDIR=/tmp
p() { n=$1; shift; timeout -k 10 200 python3 -u tools/ipm_prof.py "$@" > $O/$n.log 2>&1; r=$?; [ $r -eq 0 ] || { echo "$n rc=$r"; tail -20 $O/$n.log; exit $r; }; tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["ms_per_step"], d.get("span_us"), d.get("seg_mean_us"), d.get("seg_max_us"), d.get("critical_wave"))' $n; }
for L in 8; do
p l${L}_base 8192 $L
p l${L}_nostats 8192 $L --defs "IPM_STATS_OFF=1"
p l${L}_noxp 8192 $L --defs "IPM_XP_OFF=1"
p l${L}_none 8192 $L --defs "IPM_STATS_OFF=1;IPM_XP_OFF=1"
done
p l1_base 65536 1
p l1_nostats 65536 1 --defs "IPM_STATS_OFF=1"
p l1_noxp 65536 1 --defs "IPM_XP_OFF=1"
p l1_none 65536 1 --defs "IPM_STATS_OFF=1;IPM_XP_OFF=1"
PHGPU_FUSE_STEP=0 p l1_nofuse 65536 1
echo done
