# GPU session: parity suite, then interleaved A/B benches of variants base/cur
# (C1, then C2 when CFG2 is set). Each GPU step has its own time limit.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
VARS="${VARS:-base cur base cur}" bash tools/ab.sh || exit 1
[ -n "$CFG2" ] && CFG=$CFG2 VARS="${VARS:-base cur base cur}" bash tools/ab.sh
exit 0
