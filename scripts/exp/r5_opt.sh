# optimiser: bitwise vs the previous build (ACAMD_LIB=libacamd_base.so), unroll timing
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5opt; mkdir -p $O
B=actor_critic_algs_on_tensorflow_amd/_C/libacamd_base.so
ACAMD_LIB=$PWD/$B timeout -k 10 120 python -u scripts/exp/opt_ab.py --save $O/opt_old.pt > $O/a.log 2>&1 || { tail $O/a.log; exit 1; }
timeout -k 10 120 python -u scripts/exp/opt_ab.py --ref $O/opt_old.pt 2>&1 | tail -5
ACAMD_LIB=$PWD/$B timeout -k 10 120 python -u scripts/exp/opt_unroll_ab.py --save $O/pong_old.pt --time 400 2>&1 | tail -2
timeout -k 10 300 python -u scripts/exp/opt_unroll_ab.py --ref $O/pong_old.pt --unrolls 1,2,4,1,2,4 --time 400 2>&1 | tail -6
