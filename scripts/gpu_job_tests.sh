#!/bin/bash
# Full GPU test suite (one pytest process) + optional extra command. Usage: bash scripts/gpu_job_tests.sh TAG [pytest args]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-tests}
shift
O=gpurun_out/$TAG
mkdir -p $O
python -c "from actor_critic_algs_on_tensorflow_amd import _native; _native.load(raise_on_error=True)" || exit 3
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" $O/tests.log | tail -5; grep -E "FAILED|Error" $O/tests.log | head -20
exit $rc
