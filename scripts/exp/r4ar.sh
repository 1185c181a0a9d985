# s16 trunk forward with precomputed conv2 A-fragment bases: trunk tests, standalone A/B, instruction mix.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_r2.py tests/test_gpu_r4.py -x -q --timeout 120 --timeout-method thread -k "trunk" && \
timeout -k 10 120 python -u scripts/exp/trunk_fwd_ab.py && \
TAG=r4ar_mix bash scripts/exp/r4m.sh
