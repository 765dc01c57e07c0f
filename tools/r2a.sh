set -o pipefail
mkdir -p gpurun_out/r2a
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r2a/pytest_gpu.log 2>&1 || { echo gpu tests failed; tail -40 gpurun_out/r2a/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r2a/pytest_gpu.log
timeout -k 10 600 python -u bench.py > gpurun_out/r2a/bench.json 2> gpurun_out/r2a/bench.err || { echo bench failed; tail -20 gpurun_out/r2a/bench.err; exit 1; }
echo done
