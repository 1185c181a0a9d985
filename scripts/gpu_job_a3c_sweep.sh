#!/bin/bash
# Async-PS (GPU workers) Pendulum hyper-parameter sweep: 2 workers sharing the GPU, one line per config.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-a3csw}
mkdir -p $O
i=0
shift
for kv in "$@"; do
  i=$((i+1))
  timeout -k 10 200 python -u scripts/a3c_gpu_curve.py --workers 2 --updates 3000 --report 500 --out $O/c$i $kv > $O/c$i.log 2>&1 || { echo "fail [$kv]"; tail -5 $O/c$i.log; continue; }
  echo "[$kv] $(grep '"task": 0' $O/c$i.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print([round(r[2]) for r in d['returns']])")"
done
