set -e
mkdir -p gpurun_out
for n in ${VARS:-A B C D}; do
  RC_LIB_PATH=range_coder_rust_amd/var/librc_$n.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-adaptive --no-model-build --no-container --no-host-stream > gpurun_out/v_$n.json 2> gpurun_out/v_$n.err
  echo "$n done"
done
