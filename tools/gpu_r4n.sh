# C2 per-stage in-kernel timelines (phases per workgroup) on the current build
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TD3_LIB=tools/exp/libtd3hip_tl.so TL_DUMP=gpurun_out/tl_c2 timeout -k 10 200 python3 tools/tl_probe.py > gpurun_out/tl_c2.log 2>&1 || { tail -5 gpurun_out/tl_c2.log; exit 1; }
grep -v "amdgpu.ids" gpurun_out/tl_c2.log | head -120
SP_MODE=syncs timeout -k 10 200 python3 tools/short_probe.py > gpurun_out/sp_syncs.log 2>&1 || { tail -5 gpurun_out/sp_syncs.log; exit 1; }
grep syncs gpurun_out/sp_syncs.log
