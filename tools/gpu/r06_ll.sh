#!/bin/bash
# Round 6, pass ll: k_ph_update's grid bound (PHGPU_UPD_BLOCKS 64 / 128 / 256 / 512 / 1536) on
# config 4, by kernel trace.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6ll
mkdir -p $O
export TMPDIR=/tmp
for b in 64 128 256 512 1536; do PHGPU_UPD_BLOCKS=$b timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$b -o run -- python3 -u bench.py --model aircond --bf 32,32,64 --no-cpu-baseline --steps 10 > $O/p$b.log 2>&1 || { echo "b=$b failed"; tail -3 $O/p$b.log; exit 1; }; echo "b=$b $(grep '"k_ph_update' $O/p$b/run_kernel_stats.csv | cut -d, -f1,2,4 | cut -c1-20,100-)"; done
echo done
