#!/bin/bash
# Round 5, closing pass: the whole GPU suite and smoke(), the default bench (as the driver
# runs it), its rocprofv3 kernel trace, PMC byte and issue passes of configs 3 / 2 / 4 and the
# 8,192 share, and the other configurations' bench lines.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5f
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -2 $O/$n.log; [ $r -eq 0 ] || exit $r; }
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputests.log 2>&1
r=$?; echo "pytest rc=$r"; tail -4 $O/gputests.log; [ $r -eq 0 ] || exit $r
step smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python3 -u bench.py
step prof3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof3 -o run -- python3 -u bench.py --no-cpu-baseline
step prof2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 -u bench.py --no-cpu-baseline --scens 1024 --cm 10
echo done
