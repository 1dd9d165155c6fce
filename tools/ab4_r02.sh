set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/ab
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_scenes.py tests/test_gpu_materials.py -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_ab4.log 2>&1
rc=$?; echo "pytest rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab.sh base r01 sh2 w5
