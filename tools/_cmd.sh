set -e
V=tools/variants
timeout -k 10 200 python -u tools/ab.py --libs $V/lib_base.so $V/lib_c4.so $V/lib_c6.so $V/lib_c8.so --depths 2 --rounds 7 --out gpurun_out/ab_cap2_8k.json
timeout -k 10 200 python -u tools/ab.py --libs $V/lib_base.so $V/lib_c4.so $V/lib_c6.so $V/lib_c8.so --depths 2 --rounds 7 --images 256 --height 2160 --width 3840 --out gpurun_out/ab_cap2_4k.json
