set -e
P="python3 -c \"import json,sys; j=json.load(sys.stdin); print(j['config']['workload'][:60], j['ms_per_step'], j['roofline']['achieved'])\""
timeout -k 10 200 python -u bench.py --depth 1 --images 256 --height 2160 --width 3840 --no-cpu-baseline --no-live-pmc --no-verify | eval $P
timeout -k 10 200 python -u bench.py --config ragged --depth 1 --images 256 --height 2160 --width 3840 --ragged-min 0.999 --ragged-align 128 --steps 30 --no-cpu-baseline | eval $P
timeout -k 10 200 python -u bench.py --config ragged --depth 1 --images 256 --height 2160 --width 3840 --ragged-align 128 --steps 30 --no-cpu-baseline | eval $P
timeout -k 10 200 python -u bench.py --depth 1 --images 128 --no-cpu-baseline --no-live-pmc --no-verify | eval $P
