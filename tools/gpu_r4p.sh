# round-4 session: wide-head fix (suite + Humanoid line + tile knobs), then C2 timelines and sync costs
bash tools/gpu_r4o.sh || exit 1
bash tools/gpu_r4n.sh
