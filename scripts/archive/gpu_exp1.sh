set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/exp1
timeout -k 10 120 ./scripts/ubench_int > gpurun_out/exp1/ubench_int.txt 2>&1 || exit 1
TAG=exp1 VARIANTS="base nomac" bash scripts/gpu_exp.sh
