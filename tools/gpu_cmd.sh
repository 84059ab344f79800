set -o pipefail
F=gpurun_out/g7
mkdir -p $F
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/pytest.log 2>&1
rc=$?; tail -2 $F/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $F/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $F/smoke.log
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $F/bd.json 2> $F/bd.err; echo "bench rc=$?"
python3 -c "import json;d=json.loads(open('$F/bd.json').read().strip().splitlines()[-1]);print(d['value'], d['runs'])"
