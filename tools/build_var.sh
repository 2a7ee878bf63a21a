# build one compressor variant: tools/build_var.sh <name> <hipcc -D flags...>
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/variants
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 "$@" \
  -c ${SRC:-lz4-jpeg_amd/csrc/lz4r.hip} -o tools/variants/lz4r_$name.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -A9 "lz4_tiles" | grep -E "VGPRs:|Occupancy|LDS S" | sed "s/^.*remark: */$name: /"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/liblz4_$name.so \
  tools/variants/lz4r_$name.o $(ls lz4-jpeg_amd/build/*.o | grep -v -e "/lz4r.o" -e _seq.o -e png_io.o)
