# Driver-form warm-up effect: timed 20-step runs after 5 / 50 / 500 warm-up steps, and after 5 with
# the GPU kept busy (spin kernel) or idle (host sleep) just before the timed runs
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
set -o pipefail
for cfg in "5 none" "50 none" "500 none" "5 spin" "5 sleep" "5 none" "500 none"; do
  set -- $cfg
  WP_WARM=$1 WP_PRE=$2 timeout -k 10 120 python3 -u tools/warm_probe.py 2>/dev/null || exit 1
done
