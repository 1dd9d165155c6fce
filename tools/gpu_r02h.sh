#!/bin/bash
# Tail kernel ahead of the three-kernel bounce: full GPU suite, then the C1 A/B at the bench config.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_h.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_h.log | tail -3; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_c1full.sh base base:LUMO_TAIL=0 base:LUMO_TAIL=65536 base:LUMO_TAIL=1048576
