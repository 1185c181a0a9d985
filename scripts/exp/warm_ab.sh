# headline bench window vs warm-up length: 20 timed steps after 5 / 50 / 200 warm-up steps, and 400 after 20
set -o pipefail
O=gpurun_out/warm; mkdir -p $O
for r in 1 2; do
for w in 5 50 200; do
  timeout -k 10 150 python -u bench.py --steps 20 --warmup $w > $O/b.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "w$w $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['ms_per_step'])")"
done
done
timeout -k 10 150 python -u bench.py --steps 400 --warmup 20 > $O/b.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
echo "s400 $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['ms_per_step'])")"
