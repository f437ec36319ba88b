set -e -o pipefail
mkdir -p gpurun_out/t1
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "vs_c_oracle or aerosol or team or conservative" > gpurun_out/t1/pytest.log 2>&1 || { tail -40 gpurun_out/t1/pytest.log; exit 1; }
tail -5 gpurun_out/t1/pytest.log
