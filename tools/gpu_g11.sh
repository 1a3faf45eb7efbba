set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { tail -20 gpurun_out/bench_driver.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_driver.json'));print('driver-cmd value',d['value'],'ms',d['ms_per_step'],d['step_ms'])"
bash tools/gpu_g8.sh
