set -e
for i in 1 2; do
for combo in "0 0" "1 0" "0 1" "1 1"; do
 set -- $combo
 v=$(GSR_HOST_TOTAL=$1 GSR_BIN_GUESS=$2 timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'])")
 echo "host=$1 guess=$2 $v"
done; done
