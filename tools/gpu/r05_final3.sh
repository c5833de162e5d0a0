#!/bin/bash
# Round 5, closing pass 3: the whole GPU suite and smoke() on the final tree, the default
# bench, and the bench lines of configs 2 and 4 and of the 8,192 share.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5f3
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -2 $O/$n.log; [ $r -eq 0 ] || exit $r; }
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputests.log 2>&1
r=$?; echo "pytest rc=$r"; tail -4 $O/gputests.log; [ $r -eq 0 ] || exit $r
step smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python3 -u bench.py
step cfg2 200 python3 -u bench.py --no-cpu-baseline --scens 1024 --cm 10
step cfg4 200 python3 -u bench.py --no-cpu-baseline --model aircond
step s8192 200 python3 -u bench.py --no-cpu-baseline --scens 8192
for n in bench cfg2 cfg4 s8192; do grep '^{' $O/$n.log > $O/${n}_line.json; done
echo done
