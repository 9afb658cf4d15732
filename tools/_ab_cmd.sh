set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -m pytest tests -x -q -m gpu > gpurun_out/pytest.log 2>&1 || { tail -30 gpurun_out/pytest.log; exit 1; }
timeout -k 10 900 python tools/bench_suite.py > gpurun_out/suite.log 2>&1
