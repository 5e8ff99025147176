set -e
for sb in 8192 4096 2048 8192 4096 2048; do
WICCA_JPEG_SUB_BITS=$sb WICCA_JPEG_TIMING=1 timeout -k 10 300 python -u bench.py --config jpeg --steps 10 --no-cpu-baseline 2> gpurun_out/jpeg_sb.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$sb', d['value'], d['ms_per_step'], d['sync_rounds'], d['file_stage']['ms_per_batch'])"
tail -1 gpurun_out/jpeg_sb.err
done
