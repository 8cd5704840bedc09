# Round 4, box F: A/B of the side-stream build against HEAD and two variants,
# then the full -m gpu suite.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_ab_suite.sh r04f new base claim nhr1k sorted
