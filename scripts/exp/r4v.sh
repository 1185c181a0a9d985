# bf16-staged per-env trunk forward (mode 3): bitwise / fp32 tests, then the standalone A/B at B = 4096.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_r2.py tests/test_gpu_r4.py -x -q --timeout 120 --timeout-method thread -k "trunk" && \
timeout -k 10 120 python -u scripts/exp/trunk_fwd_ab.py
