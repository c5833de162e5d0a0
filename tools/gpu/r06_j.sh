#!/bin/bash
# Round 6, pass j: the whole GPU suite on this round's build; the loopback multi-rank step
# at the 8,192 share without the profiler.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; grep -E "passed|failed" $O/tests.log | tail -3; [ $r -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
timeout -k 10 300 python3 -u tools/fake_ranks.py 8 40 > $O/fake8.log 2>&1 && grep -E "loopback|one rank" $O/fake8.log
echo done
