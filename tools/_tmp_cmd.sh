set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r01s
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r01s/pytest.log 2>&1 || { tail -40 gpurun_out/r01s/pytest.log; exit 1; }
tail -2 gpurun_out/r01s/pytest.log
for c in config2 config3 config5; do timeout -k 10 180 python tools/profile_scan.py $c 20 || exit 1; done
timeout -k 10 180 python tools/profile_scan.py config2 50 fst || exit 1
timeout -k 10 180 python tools/profile_scan.py config3 20 fst || exit 1
