set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
GSR_BWD_WAVES=4 bash tools/gpu_wtrace.sh mt || exit 1
mkdir -p gpurun_out/driver
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/driver/bench.json 2> gpurun_out/driver/bench.err || { tail -5 gpurun_out/driver/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/driver/bench.json'));print('driver cmd', d['value'], d['ms_per_step'], d['batched']['value'])"
