# short-run anatomy: plain / gated (steps queued behind a host-released wait) / behind a sleep kernel;
# direct launches vs graph replay
set -o pipefail
for g in auto 1; do
  for m in plain gate sleep; do
    SP_MODE=$m SP_GRAPH=$g timeout -k 10 120 python3 tools/short_probe.py > gpurun_out/sp_${m}_${g}.log 2>&1 || { echo "probe $m $g failed"; tail -5 gpurun_out/sp_${m}_${g}.log; exit 1; }
    grep -v amdgpu.ids gpurun_out/sp_${m}_${g}.log
  done
done
