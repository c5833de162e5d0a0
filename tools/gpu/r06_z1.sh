#!/bin/bash
# Round 6, closing pass 1: the whole GPU suite on this round's build, then smoke().
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6z1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/ > $O/gputests.log 2>&1; r=$?; echo "tests rc=$r"; grep -E "passed|failed" $O/gputests.log | tail -2; [ $r -eq 0 ] || { grep -E "FAILED|Error" $O/gputests.log | head; exit 1; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 $O/smoke.log
echo done
