# combined: r4r (sync + suite + driver form + DP tests) then r4s (split heads)
bash tools/gpu_r4s.sh || exit 1
bash tools/gpu_r4r.sh
