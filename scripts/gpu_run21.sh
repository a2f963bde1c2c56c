set -o pipefail
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 scripts/coexec_probe.hip -o /tmp/coexec_probe 2>/dev/null || exit 4
timeout -k 10 60 /tmp/coexec_probe > gpurun_out/coexec.log 2>&1 || exit 5
echo done
