# r05 second-session evidence: scripts/gpu_profiles.sh (full GPU suite,
# smoke, bench lines, kernel traces, c2 FETCH / WRITE passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
bash scripts/gpu_profiles.sh ${OUT:-gpurun_out/r05ev2} || exit $?
echo evidence done
