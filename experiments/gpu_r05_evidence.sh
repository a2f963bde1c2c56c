# r05 evidence: scripts/gpu_profiles.sh (full GPU suite, smoke, bench lines,
# kernel traces, the c2 FETCH/WRITE passes) and the SQ counter passes of c2
# (the FC GEMMs' VALU / MFMA / LDS counts).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r05ev
bash scripts/gpu_profiles.sh $O || exit $?
CFG=c2 bash scripts/gpu_pmc_cfg.sh gpurun_out/r05ev_pmc_c2 || exit 4
python scripts/pmc_summary.py gpurun_out/r05ev_pmc_c2 > gpurun_out/r05ev_pmc_c2/summary.txt 2>&1 || true
echo evidence done
