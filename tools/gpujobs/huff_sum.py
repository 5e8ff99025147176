"""Per-call Huffman pass time (guess + sync rounds + write) from a kstats.txt."""
import sys
tot = {"guess": 0.0, "sync": 0.0, "write": 0.0}
calls = 0
for line in open(sys.argv[1]):
    f = line.split()
    if len(f) < 6 or not f[0].replace(".", "").isdigit():
        continue
    name = " ".join(f[5:])
    if "jpeg_sync_kernel<1," in name:
        tot["guess"] += float(f[0]); calls = int(f[1])
    elif "jpeg_sync_kernel<" in name:
        tot["sync"] += float(f[0])
    elif "jpeg_write_kernel" in name:
        tot["write"] += float(f[0])
n = max(calls, 1)
print(" ".join(f"{k}={v / n:.3f}" for k, v in tot.items()), f"huff={sum(tot.values()) / n:.3f}ms")
