cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python tools/latency.py 16 1024 4096 8192 16384 > gpurun_out/latency.log 2>&1 || exit 1
cat gpurun_out/latency.log
VARS="base cur base cur" bash tools/ab.sh
