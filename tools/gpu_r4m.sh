# the cleaned build: full GPU suite, then the Humanoid line
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r4m.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r4m.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --config humanoid > gpurun_out/bench_r4m_humanoid.json 2> gpurun_out/bench_r4m_humanoid.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/bench_r4m_humanoid.json'));print('humanoid',d['value'],d['runs'],d['roofline']['traffic'])"
