# Host wait mode of the end-of-run sync (hipSetDeviceFlags) in the driver's 20-step form
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
set -o pipefail
for spin in "" pre pre:4 post post:4; do
  SP_SPIN=$spin timeout -k 10 120 python3 -u tools/short_probe.py > gpurun_out/r4x_spin_${spin/:/_}.txt 2>&1 || { echo "probe $spin failed"; tail gpurun_out/r4x_spin_${spin/:/_}.txt; exit 1; }
  echo "== SP_SPIN=$spin"; grep -E "hipSet|run [0-7]|per train" gpurun_out/r4x_spin_${spin/:/_}.txt
done
