# build one JPEG-kernel variant: tools/build_jvar.sh <name> <hipcc -D flags...>
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/variants
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 "$@" \
  -c lz4-jpeg_amd/csrc/jpegr.hip -o tools/variants/jpegr_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/liblz4_$name.so \
  tools/variants/jpegr_$name.o $(ls lz4-jpeg_amd/build/*.o | grep -v -e "/jpegr.o" -e _seq.o -e png_io.o)
