set -e
mkdir -p gpurun_out/r06n
for v in c16 tight f64a; do
  echo "== $v" >> gpurun_out/r06n/probe.txt
  HD_LIB_PATH=$PWD/mb/$v/libhdisort.so timeout -k 10 300 python scripts/micro/probe_solve.py mb/worst_c16.npz 2>/dev/null | head -3 >> gpurun_out/r06n/probe.txt
done
