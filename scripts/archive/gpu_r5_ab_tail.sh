set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/tail; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/suite.log 2>&1 || exit 1
A="--no-cpu-baseline --no-host-path --no-prove --sustain-seconds 0"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --config c2 $A > $O/c2_tail_$i.log 2>&1 || exit 1
  HB_LIB_PATH=$PWD/exp_notail.so timeout -k 10 200 python -u bench.py --config c2 $A > $O/c2_notail_$i.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 $A > $O/c3_tail_$i.log 2>&1 || exit 1
  HB_LIB_PATH=$PWD/exp_notail.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 $A > $O/c3_notail_$i.log 2>&1 || exit 1
done
echo ok
