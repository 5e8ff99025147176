set -e
V=tools/variants
timeout -k 10 300 python -u tools/ab.py --libs $V/lib_base.so $V/lib_mw2.so --multi 1,2,3,4,5,6 --rounds 5 --out gpurun_out/ab_k5_mw16.json
timeout -k 10 300 python -u tools/ab.py --libs $V/lib_base.so $V/lib_mw2.so --multi 2,3,4,5,6 --rounds 5 --out gpurun_out/ab_k5_mw26.json
