set -o pipefail
F=gpurun_out/g6
mkdir -p $F
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/pytest.log 2>&1
rc=$?; tail -4 $F/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for v in 1 0; do
TD3_L0R16_N112=$v timeout -k 10 200 python3 bench.py --steps 2000 --warmup 100 --no-cpu-baseline --no-roofline > $F/b_${v}_$i.json 2> $F/b_${v}_$i.err || exit 1
python3 -c "import json;d=json.loads(open('$F/b_${v}_$i.json').read().strip().splitlines()[-1]);print('n112=$v', d['value'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $F/prof -o run -- python3 bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-roofline > $F/prof.log 2>&1; echo "prof rc=$?"
grep -E "l0r16|gemm_kernel<0, 2, 5>" $F/prof/run_kernel_stats.csv | cut -c1-120
