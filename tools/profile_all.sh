# rocprofv3 kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes for every bench preset.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-r01j}
for c in c3 c5 c1 c2; do
  bash "$R/tools/profile.sh" ${TAG}_$c --config $c --steps 3
done
