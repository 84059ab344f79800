# Deferred online-actor layer 2 (TF_fwd2) + pi(s) head in the critic_loss launch: every -m gpu
# test on the new build, then C2 / Humanoid A/B against the round-3 layout (TD3_DEFER_ACTOR_L2=0)
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
set -o pipefail
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r4ae.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r4ae.log; [ $rc -ne 0 ] && { grep -E "FAILED|ERROR|Error" gpurun_out/pytest_r4ae.log | head; exit $rc; }
L=tools/exp/libtd3hip_nodefer.so
for lib in $L td3_amd/libtd3hip.so $L td3_amd/libtd3hip.so; do
  TD3_LIB=$lib timeout -k 10 200 python3 bench.py --steps 2000 --warmup 100 --runs 3 --no-cpu-baseline > gpurun_out/r4ae.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r4ae.json'));s=d['stage_us'];print('$lib', d['value'], {k:v for k,v in s.items() if k.startswith('1:') and k[2:] in ('F_fwd2','heads','CB_bwd1+TF_fwd2','critic_loss','TF_fwd2')})"
done
for lib in $L td3_amd/libtd3hip.so $L td3_amd/libtd3hip.so; do
  TD3_LIB=$lib timeout -k 10 200 python3 bench.py --config humanoid --steps 600 --warmup 50 --runs 3 --no-cpu-baseline > gpurun_out/r4ae_h.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r4ae_h.json'));s=d['stage_us'];print('humanoid $lib', d['value'], {k:v for k,v in s.items() if k.startswith('1:') and k[2:] in ('F_fwd2','heads','TF_fwd2','critic_loss')})"
done
