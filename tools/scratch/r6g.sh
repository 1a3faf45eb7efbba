#!/bin/bash
# split SH preprocess: stream modes A/B on the metric bench
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6g; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "c1_config or sh3" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for m in 0 1 2 3 4; do
    GSR_SH_SPLIT=$m timeout -k 10 300 python bench.py --steps 200 --no-cpu-baseline --no-train --stages > $O/mt_${m}_$i.json 2> $O/mt_${m}_$i.err || { tail -5 $O/mt_${m}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$O/mt_${m}_$i.json'));print('mode=$m', d['value'], d['ms_per_step'], d.get('batched',{}).get('value'), ' '.join('%s=%.4f'%(k,v['avg_ms']) for k,v in d['stages'].items()))"
  done
done
