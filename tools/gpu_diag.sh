cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() { n=$1; echo "== $n"; shift; env "$@" timeout -k 10 120 python3 tools/grad_diag.py > gpurun_out/diag_$n.log 2>&1; grep -E "^step|BAD|tile max|^    |worst" gpurun_out/diag_$n.log | head -40; }
run map DIAG_MAP=1
run odd2 DIAG_ODD2=1
run dwsk0 TD3_LIB=tools/exp/libtd3hip_dwsk0.so
