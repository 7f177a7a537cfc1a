set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
LIBS="dual cur" WLS="config4" STEPS=4 BENCH_EXTRA="--envs 262144" tools/gpu_ab.sh r04h_e262144 || exit 1
