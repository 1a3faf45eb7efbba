set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for so in "" build/variants/libgsr_*.so; do
  if [ -n "$so" ]; then export GSR_LIBRARY=$PWD/$so; else unset GSR_LIBRARY; fi
  timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -x -q -k "large_gaussians or depth_sort_grouped or c1_config" --timeout 60 --timeout-method thread > gpurun_out/bis.log 2>&1
  echo "== ${so:-default}: $(tail -1 gpurun_out/bis.log)"
done
