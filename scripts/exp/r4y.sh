# Row-split fused step with the head's loads first: bitwise tests, phase stamps, headline bench.
set -o pipefail
O=gpurun_out/${TAG:-r4y}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_r2.py tests/test_gpu_r4.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "fused or trunk or rows" && \
timeout -k 10 300 python -u scripts/exp/rows_step_phases.py > $O/phases.json && cat $O/phases.json && \
timeout -k 10 300 python -u bench.py --steps 400 --warmup 20
