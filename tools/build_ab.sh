# Build an A/B variant of the compressor from a copy of lz4r.hip:
#   tools/build_ab.sh path/to/lz4r.hip name  ->  tools/variants/liblz4_<name>.so
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/variants
cp "$1" tools/variants/lz4r_$2.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 $EXTRA \
  -I include -c tools/variants/lz4r_$2.hip -o tools/variants/lz4r_$2.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/liblz4_$2.so \
  tools/variants/lz4r_$2.o $(ls lz4-jpeg_amd/build/*.o | grep -v -e "/lz4r.o" -e _seq.o -e _par.o -e png_io.o)
