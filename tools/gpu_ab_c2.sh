set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ckn; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash tools/ab_kstats.sh 2 > $O/ab_mt.log 2>&1 || { tail -20 $O/ab_mt.log; exit 1; }
cat $O/ab_mt.log
CONFIG=c2 bash tools/ab_kstats.sh 2 > $O/ab_c2.log 2>&1 || { tail -20 $O/ab_c2.log; exit 1; }
cat $O/ab_c2.log
