# Build of the MI355X base64 byte-stream engine and its test oracle.
#
#   make            -> async_amd/libasync_b64.so  (product: HIP kernels + C ABI
#                      + bytestream_1 stages + minimal loop/streams)
#                      oracle/liboracle.so          (test infrastructure only)
#                      tests/csrc/libstage_harness.so, libstage_fake.so,
#                      libb64x_hooks.so     (test infrastructure only)
#   make clean
#
# Everything is compiled for gfx950 only (no other offload targets, no
# CUDA/HIP dual path).  Code object v5 keeps the library loadable by both
# the ROCm 7.2 runtime of this image and the ROCm 7.0 runtime bundled with
# the PyTorch wheel (the Python side imports torch first, see
# async_amd/_lib.py).

HIPCC    ?= /opt/rocm/bin/hipcc
CC       ?= gcc
ARCH     ?= gfx950
# -Wno-pass-failed: k_encode_flat's `#pragma unroll` loops (compile-time trip
# counts) are reported "not unrolled" after they have already been fully
# unrolled by an earlier pass; the ISA is the unrolled one.
# -amdgpu-kernarg-preload-count: the first 16 dwords of kernel arguments
# arrive in SGPRs, so a wave's first address needs no kernarg load (encode
# -2 us, CRLF-76 decode -2.5 us per 1 GiB in A/B; the code object keeps the
# loading prologue for firmware without preload).
HIPFLAGS  = --offload-arch=$(ARCH) -mcode-object-version=5 -O3 -std=c++17 -fPIC -Iasync_amd/csrc \
            -Wall -Wno-pass-failed -Iinclude -mllvm -amdgpu-kernarg-preload-count=16
CFLAGS    = -O2 -std=c11 -fPIC -Wall -Wextra -Wno-unused-parameter -Iinclude

LIB      = async_amd/libasync_b64.so
# Stages + kernels only (no event loop/streams/allocator): the drop-in for a
# build of the reference library, which supplies async_wound(), the streams
# and (through fsdyn) fsalloc()/fsfree().
CORE     = async_amd/libasync_b64_core.so
ORACLE   = oracle/liboracle.so
HARNESS  = tests/csrc/libstage_harness.so
OBJDIR   = build

KERNEL_SRC = async_amd/csrc/b64x_kernels.hip
HOST_SRC   = async_amd/csrc/fsalloc.c async_amd/csrc/loop.c async_amd/csrc/streams.c \
             async_amd/csrc/framing.c async_amd/csrc/fdstreams.c async_amd/csrc/b64_hub.c \
             async_amd/csrc/b64_stages.c async_amd/csrc/b64_pin.c
HEADERS    = $(wildcard include/*.h)

HOST_OBJ   = $(patsubst async_amd/csrc/%.c,$(OBJDIR)/%.o,$(HOST_SRC))

# The same harness over the product's host C with a CPU stand-in for the GPU
# side (tests/csrc/fake_b64x.c): deterministic, adversarially ordered tests
# of the stages' slot accounting, no GPU needed (test infrastructure only).
FAKE     = tests/csrc/libstage_fake.so
# The kernels again with the test-only hooks compiled in (B64X_TEST_HOOKS:
# forced decode range lengths); never linked into the product libraries.
HOOKS    = tests/csrc/libb64x_hooks.so

all: $(LIB) $(CORE) $(ORACLE) $(HARNESS) $(FAKE) $(HOOKS)

$(OBJDIR):
	mkdir -p $(OBJDIR)

$(OBJDIR)/b64x_kernels.o: $(KERNEL_SRC) $(HEADERS) async_amd/csrc/b64x_result_check.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.o: async_amd/csrc/%.c $(HEADERS) async_amd/csrc/b64_hub.h async_amd/csrc/b64_lend.h async_amd/csrc/b64_pin.h | $(OBJDIR)
	$(CC) $(CFLAGS) -c $< -o $@

$(OBJDIR)/b64x_kernels_hooks.o: $(KERNEL_SRC) $(HEADERS) async_amd/csrc/b64x_result_check.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -DB64X_TEST_HOOKS -c $< -o $@

$(HOOKS): $(OBJDIR)/b64x_kernels_hooks.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^ -Wl,-soname,libb64x_hooks.so

$(LIB): $(OBJDIR)/b64x_kernels.o $(HOST_OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^ -Wl,-soname,libasync_b64.so

$(CORE): $(OBJDIR)/b64x_kernels.o $(OBJDIR)/b64_hub.o $(OBJDIR)/b64_stages.o $(OBJDIR)/b64_pin.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^ -Wl,-soname,libasync_b64_core.so

$(ORACLE): oracle/b64_oracle.c oracle/b64_oracle.h
	$(CC) -O2 -std=c11 -fPIC -Wall -Wextra -shared -o $@ oracle/b64_oracle.c

$(HARNESS): tests/csrc/stage_harness.c $(LIB) $(HEADERS)
	$(CC) $(CFLAGS) -shared -o $@ tests/csrc/stage_harness.c \
	    -Lasync_amd -lasync_b64 -Wl,-rpath,'$$ORIGIN/../../async_amd' \
	    -L/opt/rocm/lib -lamdhip64 -lpthread

$(FAKE): tests/csrc/stage_harness.c tests/csrc/fake_b64x.c oracle/b64_oracle.c $(HOST_SRC) $(HEADERS) \
         async_amd/csrc/b64_hub.h async_amd/csrc/b64_lend.h async_amd/csrc/b64x_result_check.h
	$(CC) $(CFLAGS) -Ioracle -Iasync_amd/csrc -shared -o $@ tests/csrc/stage_harness.c \
	    tests/csrc/fake_b64x.c oracle/b64_oracle.c $(HOST_SRC) -lpthread

clean:
	rm -rf $(OBJDIR) $(LIB) $(CORE) $(ORACLE) $(HARNESS) $(FAKE) $(HOOKS)

.PHONY: all clean

