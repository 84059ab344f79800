cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for o in 1 0; do
  echo "== TD3_DWSK_ORDER=$o"
  TD3_DWSK_ORDER=$o timeout -k 10 120 python3 tools/grad_diag.py 2>&1 | grep -E "step|BAD" | head -30
done
echo "== DIAG_B=512 order 1"
DIAG_B=512 timeout -k 10 120 python3 tools/grad_diag.py 2>&1 | grep -E "step|BAD" | head -20
