#!/bin/bash
# C++ autograd route: its tests, the API / multi-view / host tests it touches, host overhead per
# route, and the C1 / mt bench lines
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6e; rm -rf $O; mkdir -p $O
: pytest done

for cfg in; do
  timeout -k 10 300 python tools/host_overhead.py $cfg 300 > $O/host_${cfg}.txt 2>&1 || { tail -20 $O/host_${cfg}.txt; exit 1; }
  GSR_HOST_AUTOGRAD=0 timeout -k 10 300 python tools/host_overhead.py $cfg 300 > $O/host_${cfg}_pyfn.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/host_*.txt
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --config c1 --steps 200 --warmup 20 --no-cpu-baseline --no-train --batched-views 1 > $O/c1_$i.json 2> $O/c1_$i.err || { tail -5 $O/c1_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c1_$i.json'));print('c1', d['value'], d['ms_per_step'])"
done
GSR_HOST_AUTOGRAD=0 timeout -k 10 300 python bench.py --config c1 --steps 200 --warmup 20 --no-cpu-baseline --no-train --batched-views 1 > $O/c1_pyfn.json 2> $O/c1_pyfn.err || exit 1
python -c "import json;d=json.load(open('$O/c1_pyfn.json'));print('c1 pyfn', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --steps 200 --no-cpu-baseline --no-train > $O/mt.json 2> $O/mt.err || { tail -5 $O/mt.err; exit 1; }
python -c "import json;d=json.load(open('$O/mt.json'));print('mt', d['value'], d['ms_per_step'], d.get('batched',{}).get('value'))"
