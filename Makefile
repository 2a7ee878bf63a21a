# Build everything for MI355X (gfx950).  `make -j8` in the build container
# cross-compiles; the built .so / executables travel to the GPU box in-tree.
#
#   lz4-jpeg_amd/lz4jpeg/liblz4jpeg.so   product C-ABI library (HIP kernels)
#   lz4-jpeg_amd/bin/LZ4_seq, JPEG_seq    drop-in executables (file contract)
#   oracle/liboracle.so (+ oracle/_ref)   test-only CPU checker
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
CC      ?= gcc
PKG     := lz4-jpeg_amd
CSRC    := $(PKG)/csrc
HIPFLAGS := --offload-arch=$(ARCH) -O3 -ffp-contract=off -fPIC -std=c++17 -Wall \
            -Wno-unused-result
LIB     := $(PKG)/lz4jpeg/liblz4jpeg.so
HIP_SRC := $(CSRC)/lz4r.hip $(CSRC)/jpegr.hip
HDRS    := include/lz4r.h include/jpegr.h $(CSRC)/jpeg_tables.h

all: lib oracle

lib: $(LIB)

$(CSRC)/jpeg_tables.h: $(CSRC)/gen_jpeg_tables.py
	python3 $< > $@

$(PKG)/build/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(PKG)/build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(PKG)/build/synth.o: $(PKG)/host/synth.c
	@mkdir -p $(PKG)/build
	$(CC) -O2 -fPIC -Wall -c $< -o $@

$(LIB): $(PKG)/build/lz4r.o $(PKG)/build/jpegr.o $(PKG)/build/synth.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(PKG)/build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all lib oracle clean
