#!/bin/bash
# shared-matrix streaming path: first check (aircond parity vs default path, UC vs HiGHS)
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/stream_check.py aircond > gpurun_out/stream_aircond.log 2>&1
rc=$?; echo "aircond rc=$rc"; tail -8 gpurun_out/stream_aircond.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/stream_check.py uc 4 > gpurun_out/stream_uc.log 2>&1
rc=$?; echo "uc rc=$rc"; tail -8 gpurun_out/stream_uc.log
exit $rc
