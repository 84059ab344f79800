cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() { echo "== $1"; shift; env "$@" timeout -k 10 120 python3 tools/grad_diag.py 2>&1 | grep -v "^  critic s.*[0-9]$" | head -40; }
run map DIAG_MAP=1
run odd2 DIAG_ODD2=1
run dwsk0 TD3_LIB=tools/exp/libtd3hip_dwsk0.so
