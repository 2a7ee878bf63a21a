# Build everything for MI355X (gfx950).  `make -j8` in the build container
# cross-compiles; the built .so / executables travel to the GPU box in-tree.
#
#   lz4-jpeg_amd/lz4jpeg/liblz4jpeg.so   product C-ABI library (HIP kernels)
#   lz4-jpeg_amd/bin/LZ4_seq, JPEG_seq    drop-in executables (file contract),
#                                         also as LZ4_seq.exe / JPEG_seq.exe
#   oracle/liboracle.so (+ oracle/_ref)   test-only CPU checker
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
CC      ?= gcc
PKG     := lz4-jpeg_amd
CSRC    := $(PKG)/csrc
HOST    := $(PKG)/host
B       := $(PKG)/build
BIN     := $(PKG)/bin
HIPFLAGS := --offload-arch=$(ARCH) -O3 -ffp-contract=off -fno-strict-aliasing -fPIC -std=c++17 -Wall \
            -Wno-unused-result
# lz4r.hip (the compressor): the max-ILP machine scheduler, -0.3 % lz4_tiles and
# call time in three in-process A/B orders (tools/ab_inproc.py)
LZ4R_HIPFLAGS := -mllvm -amdgpu-sched-strategy=max-ilp
CFLAGS_HOST := -O2 -fPIC -Wall -std=gnu11 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include
LIB     := $(PKG)/lz4jpeg/liblz4jpeg.so
HDRS    := include/lz4r.h include/jpegr.h include/lz4jpeg_compat.h include/lz4jpeg_synth.h \
           $(CSRC)/jpeg_tables.h
OBJS    := $(B)/lz4r.o $(B)/lz4r_gpudec.o $(B)/jpegr.o $(B)/jpegr_blocks.o $(B)/jpegr_entropy.o \
           $(B)/synth.o $(B)/synth_dev.o \
           $(B)/lz4r_decode.o $(B)/compat.o $(B)/compat_lz4.o

all: lib bin oracle tools

lib: $(LIB)

bin: $(BIN)/LZ4_seq $(BIN)/JPEG_seq $(BIN)/LZ4_seq.exe $(BIN)/JPEG_seq.exe \
     $(BIN)/LZ4_par $(BIN)/JPEG_par $(BIN)/LZ4_par.exe $(BIN)/JPEG_par.exe

$(CSRC)/jpeg_tables.h: $(CSRC)/gen_jpeg_tables.py
	python3 $< > $@

$(B)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(B)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(B)/lz4r.o: HIPFLAGS += $(LZ4R_HIPFLAGS)
# the block decoder: the max-memory-clause scheduler, -0.45 % (tools/ab_dec_inproc.py)
$(B)/lz4r_gpudec.o: HIPFLAGS += -mllvm -amdgpu-sched-strategy=max-memory-clause

$(B)/%.o: $(HOST)/%.c $(HDRS) $(HOST)/lzj_host.h
	@mkdir -p $(B)
	$(CC) $(CFLAGS_HOST) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

# executables link the objects statically (no liblz4jpeg.so lookup at run time)
$(BIN)/LZ4_seq: $(B)/lz4_seq.o $(OBJS)
	@mkdir -p $(BIN)
	$(HIPCC) --offload-arch=$(ARCH) -o $@ $^

$(BIN)/JPEG_seq: $(B)/jpeg_seq.o $(B)/png_io.o $(OBJS)
	@mkdir -p $(BIN)
	$(HIPCC) --offload-arch=$(ARCH) -o $@ $^ -lz

# the parallel drivers' executables (Experiment/*_parallel_experiment.c)
$(B)/lz4_par.o: $(HOST)/lz4_seq.c $(HDRS)
	@mkdir -p $(B)
	$(CC) $(CFLAGS_HOST) -DLZ4_PAR -c $< -o $@

$(BIN)/LZ4_par: $(B)/lz4_par.o $(OBJS)
	@mkdir -p $(BIN)
	$(HIPCC) --offload-arch=$(ARCH) -o $@ $^

$(BIN)/JPEG_par: $(BIN)/JPEG_seq
	cp $< $@

$(BIN)/%.exe: $(BIN)/%
	cp $< $@

oracle:
	$(MAKE) -C oracle

# ASan + UBSan build of the host C (no HIP) and the oracle restatements,
# driven by tests/sanitize/sanitize_main.c; tests/test_sanitize.py
SAN_SRC := tests/sanitize/sanitize_main.c tests/sanitize/cpu_matches.c $(HOST)/lz4r_decode.c \
           $(HOST)/png_io.c $(HOST)/synth.c $(HOST)/compat_lz4.c \
           oracle/lz4_oracle.c oracle/jpeg_oracle.c oracle/jpeg_entropy_oracle.c
sanitize: build/sanitize_main

build/sanitize_main: $(SAN_SRC) include/lz4r.h include/lz4jpeg_synth.h include/lz4jpeg_compat.h \
                     $(HOST)/lzj_host.h
	@mkdir -p build
	$(CC) -O1 -g -std=gnu11 -ffp-contract=off -fno-omit-frame-pointer \
	  -fsanitize=address,undefined -fno-sanitize-recover=all \
	  -o $@ $(SAN_SRC) -lz -lm -lpthread

# micro-benchmarks: SIMD issue rates (tools/issue.sh) and LDS access costs
tools: tools/variants/valu_rate tools/variants/lds_rate

tools/variants/valu_rate: tools/valu_rate.hip
	@mkdir -p tools/variants
	$(HIPCC) --offload-arch=$(ARCH) -O3 -o $@ $<

tools/variants/lds_rate: tools/lds_rate.hip
	@mkdir -p tools/variants
	$(HIPCC) --offload-arch=$(ARCH) -O3 -Wno-unused-result -o $@ $<

clean:
	rm -rf $(B) $(BIN) $(LIB) build
	$(MAKE) -C oracle clean

.PHONY: all lib bin oracle tools sanitize clean

# `make -s print-HIPFLAGS`: a variable's value (tests/test_isa.py builds with the product flags)
print-%:
	@echo $($*)
