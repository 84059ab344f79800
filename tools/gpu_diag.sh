cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() { echo "== $1"; shift; env "$@" timeout -k 10 120 python3 tools/grad_diag.py 2>&1 | grep -E "step 2|BAD" | head -8; }
run base X=1
run wn4x2off TD3_LIB=tools/exp/libtd3hip_wn4x2off.so
run unitoff TD3_LIB=tools/exp/libtd3hip_unitoff.so
run wn2bwd0 TD3_WN2_BWD=0
run wn4min0 TD3_WN4_MIN=0
run graphoff TD3_DIAG_EAGER=1
