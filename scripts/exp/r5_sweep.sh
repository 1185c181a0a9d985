# headline EngineOpts sweep at 400 steps, two rounds: OPTS="json1;json2;..."
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5sweep; mkdir -p $O
IFS=';' read -ra LIST <<< "$OPTS"
for r in 1 2; do
for eo in "${LIST[@]}"; do
  timeout -k 10 150 python -u bench.py --steps 400 --warmup 20 --engine-opts "$eo" > $O/b.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "$eo $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['ms_per_step'])")"
done
done
