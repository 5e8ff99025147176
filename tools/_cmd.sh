set -e
V=tools/variants
A="--libs $V/lib_base.so $V/lib_flat.so --depths 2 3 --rounds 7 --images 256 --height 2160 --width 3840"
timeout -k 10 200 python -u tools/ab.py $A --out gpurun_out/ab_flat2_uni.json
timeout -k 10 200 python -u tools/ab.py $A --ragged 1.0 --ragged-align 128 --out gpurun_out/ab_flat2_rag10.json
timeout -k 10 200 python -u tools/ab.py $A --ragged 0.5 --ragged-align 128 --out gpurun_out/ab_flat2_rag05.json
