set -o pipefail
F=gpurun_out/g2
mkdir -p $F
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/pytest.log 2>&1
rc=$?; tail -2 $F/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ko.sh st0
