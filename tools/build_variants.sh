# Build timing-ablation variants of liblz4jpeg.so into tools/variants/ (not shipped).
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/variants
for v in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-strict-aliasing -fPIC -std=c++17 $EXTRA -DLZ4R_VARIANT=$v \
    -c lz4-jpeg_amd/csrc/lz4r.hip -o tools/variants/lz4r_v$v.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/liblz4_v$v.so \
    tools/variants/lz4r_v$v.o $(ls lz4-jpeg_amd/build/*.o | grep -v -e "/lz4r.o" -e _seq.o -e png_io.o)
done
# profiled builds: PROF="0 1" -> liblz4_p0.so, liblz4_p1.so (LZ4R_PROF + variant)
for v in $PROF; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-strict-aliasing -fPIC -std=c++17 -DLZ4R_PROF -DLZ4R_VARIANT=$v \
    -c lz4-jpeg_amd/csrc/lz4r.hip -o tools/variants/lz4r_p$v.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/liblz4_p$v.so \
    tools/variants/lz4r_p$v.o $(ls lz4-jpeg_amd/build/*.o | grep -v -e "/lz4r.o" -e _seq.o -e png_io.o)
done
