mkdir -p gpurun_out
set -e
timeout -k 5 60 ./tools/micro/wave_lat > gpurun_out/wave_lat.txt 2>&1

timeout -k 5 30 ./tools/micro/dpp_check > gpurun_out/dpp.txt 2>&1
for w in "" --c3 --e2e; do
  GPUSCHED_LIB=libgpusched_tl.so timeout -k 10 150 python3 tools/ffd_diag.py $w --tl >> gpurun_out/tl_base.txt 2>&1
done
timeout -k 10 120 python3 tools/ffd_diag.py >> gpurun_out/tl_base.txt 2>&1
