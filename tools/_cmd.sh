set -e
V=tools/variants
A="--libs $V/lib_cur.so $V/lib_rcap4.so $V/lib_rcap6.so $V/lib_strip.so --depths 1 3 --rounds 5 --images 256 --height 2160 --width 3840 --ragged-align 128"
timeout -k 10 150 python -u tools/ab.py $A --ragged 1.0 --out gpurun_out/ab_rcap_r10.json | sed 's/^/r1.0 /'
timeout -k 10 150 python -u tools/ab.py $A --ragged 0.5 --out gpurun_out/ab_rcap_r05.json | sed 's/^/r0.5 /'
