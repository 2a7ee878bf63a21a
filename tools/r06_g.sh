# round 6: lz4_emit phase ablations (outputs wrong except v0; only times count):
# 31 no literal words, 32 no header bytes, 33 no records->bytes phase,
# 34 no image->stream stores, 35 no image zeroing, 37 = 33 + 34 (loads, staging, offsets)
set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
A=tools/ab
timeout -k 10 400 python -u tools/ab_inproc.py 20 $A/liblz4_v0.so $A/liblz4_v31.so $A/liblz4_v32.so $A/liblz4_v33.so $A/liblz4_v34.so $A/liblz4_v35.so $A/liblz4_v37.so $A/liblz4_v0.so > $O/emit_ablate.log 2>&1
