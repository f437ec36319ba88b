set -e -o pipefail
mkdir -p gpurun_out/r06p
HD_LIB_PATH=$PWD/mb/pol/libhdisort.so timeout -k 10 400 python scripts/micro/find_worst.py gpurun_out/r06p/worst_pol.npz > gpurun_out/r06p/full_c4_pol.txt 2>&1
timeout -k 10 400 python scripts/micro/find_worst.py gpurun_out/r06p/worst_c5.npz 0 64 0 c5 > gpurun_out/r06p/full_c5.txt 2>&1
bash scripts/ab/c4_ab.sh r06p sc pol sc pol
