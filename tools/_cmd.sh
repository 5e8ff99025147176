set -e
V=tools/variants
timeout -k 10 300 python -u tools/ab.py --libs $V/lib_base.so $V/lib_cap6.so $V/lib_cap0.so $V/lib_x64.so --depths 3 --rounds 7 --steps 30 --images 32 --height 2160 --width 3840 --out gpurun_out/ab_4k_d3.json
