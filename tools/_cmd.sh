set -e
V=tools/variants
for rep in 1 2; do for v in stage1 stage0; do
WICCA_HIP_LIB=$V/lib_$v.so WICCA_JPEG_TIMING=1 timeout -k 10 300 python -u bench.py --config jpeg --steps 10 --no-cpu-baseline 2> gpurun_out/jpeg_$v.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['file_stage']['ms_per_batch'])"
tail -1 gpurun_out/jpeg_$v.err
done; done
