# final check of the committed tree's library: GPU suite and smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06z
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r06z/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06z/smoke.log 2>&1
tail -n 1 gpurun_out/r06z/pytest_gpu.log; cat gpurun_out/r06z/smoke.log | tail -n 1
