#!/bin/bash
# split SH preprocess: parity, A/B of the metric bench, kernel trace
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6f; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_host_autograd.py tests/test_gpu_multiview.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  for split in 1 0; do
    GSR_SH_SPLIT=$split timeout -k 10 300 python bench.py --steps 200 --no-cpu-baseline --no-train --stages > $O/mt_${split}_$i.json 2> $O/mt_${split}_$i.err || { tail -5 $O/mt_${split}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$O/mt_${split}_$i.json'));print('split=$split', d['value'], d['ms_per_step'], d.get('batched',{}).get('value'), ' '.join('%s=%.4f'%(k,v['avg_ms']) for k,v in d['stages'].items()))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-train --batched-views 1 > $O/prof.json 2> $O/prof.log || { tail -20 $O/prof.log; exit 1; }
cp $(find $O/prof -name "*kernel_trace.csv" | head -1) $O/kernel_trace.csv
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
python tools/kstats.py $O/kernel_stats.csv | head -12
