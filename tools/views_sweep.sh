cd /root/repo; mkdir -p gpurun_out
for b in 1 2 4 8; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-train --views-per-gpu $b --batched-views 1 --steps 40 --warmup 4 > gpurun_out/vb$b.json 2> gpurun_out/vb$b.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/vb$b.json'));print($b, d['value'], {k:round(v['avg_ms']*1e3,1) for k,v in d['stages'].items()})"
done
