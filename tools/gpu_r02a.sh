#!/bin/bash
# Round-2 GPU pass A (repo root on the GPU box): all GPU parity tests (incl. the full-scale C2/C3
# and kernel-variant matrix), smoke, the default bench (C1 + C3 Bistro @256 spp), C3 rocprofv3
# trace + FETCH/WRITE passes, and the 8-B/lane PMC calibration.  Test assertion failures (rc 1)
# do not stop the later steps; any other failure (fault, abort, time limit) ends the script.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
timeout -k 10 900 python3 bench.py --steps 3 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err
bash tools/profile.sh r02a_c3 --config c3 --spp 8 --steps 1 --warmup 0 --cpu-baseline 0
bash tools/calib.sh
echo done
