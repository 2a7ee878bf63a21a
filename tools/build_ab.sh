# Build an A/B variant library from a modified copy of one product source:
#   tools/build_ab.sh path/to/file.hip name [lz4r|jpegr|...]
#     -> tools/ab/lib<obj>_<name>.so  (the product objects, with
#        build/<obj>.o replaced by the variant; default obj: lz4r, lib prefix
#        liblz4_ for lz4r and libjpeg_ for jpegr)
set -e
cd "$(dirname "$0")/.."
obj=${3:-lz4r}
case $obj in lz4r) lib=liblz4_$2.so ;; jpegr) lib=libjpeg_$2.so ;; *) lib=lib${obj}_$2.so ;; esac
mkdir -p tools/ab
cp "$1" tools/ab/${obj}_$2.hip
[ $obj = lz4r ] && [ -z "$NO_LZ4R_FLAGS" ] && EXTRA="$EXTRA $(make -s print-LZ4R_HIPFLAGS)"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-strict-aliasing -fPIC -std=c++17 $EXTRA \
  -I include -I lz4-jpeg_amd/csrc -c tools/ab/${obj}_$2.hip -o tools/ab/${obj}_$2.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/ab/$lib \
  tools/ab/${obj}_$2.o $(ls lz4-jpeg_amd/build/*.o | grep -v -e "/$obj.o" -e _seq.o -e _par.o -e png_io.o)
echo built tools/ab/$lib
