set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_generate.py -k "steps_per_replay or streams or beam" > gpurun_out/r03al_pytest.txt 2>&1; rc=$?; tail -20 gpurun_out/r03al_pytest.txt | grep -E "PASS|FAIL|passed|failed"; [ $rc -eq 0 ] &&
timeout -k 10 400 python -u tools/lab/replay_k.py > gpurun_out/r03al_replay_k.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r03al_replay_k.txt | tail -10; exit $rc
