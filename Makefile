# Build of the MI355X reduction engine (libnccl.so, C ABI of include/nccl.h) and of the CPU oracle.
#   make            -> nccl_amd/lib/libnccl.so  +  oracle/_build/liboracle.so
#   make lib        -> only the product library
#   make oracle     -> only the test oracle
HIPCC    ?= /opt/rocm/bin/hipcc
CXX      := /opt/rocm/lib/llvm/bin/clang++
ARCH     ?= gfx950
BUILD    := build
LIBDIR   := nccl_amd/lib
SRCDIR   := nccl_amd/csrc

# -ffp-contract=off: never fuse x*s + acc into one FMA (PreMulSum parity).
# -fno-gpu-flush-denormals-to-zero: keep fp32 denormals like the reference (no -ftz, common.mk:103).
# EXTRA: extra defines for A/B builds of variants (e.g. EXTRA=-DNCCL_AMD_COPY_UNROLL=16 BUILD=build_ab LIBDIR=ablib/x)
EXTRA    ?=
COMMON   := -O3 -fPIC -std=c++17 -ffp-contract=off -fvisibility=hidden -Wall -Wno-unused-function \
            -Wno-unused-variable -Wno-unused-but-set-variable -Iinclude $(EXTRA)
HIPFLAGS := $(COMMON) --offload-arch=$(ARCH) -fno-gpu-flush-denormals-to-zero -munsafe-fp-atomics
HOSTSRC  := debug.cc bootstrap.cc ipc.cc transport.cc init.cc group.cc enqueue.cc register.cc tuner.cc mapcheck.cc
HOSTOBJ  := $(HOSTSRC:%.cc=$(BUILD)/%.o)
DEVSRC   := $(notdir $(wildcard $(SRCDIR)/*.hip))
DEVOBJ   := $(DEVSRC:%.hip=$(BUILD)/%.o)
HDRS     := $(wildcard $(SRCDIR)/*.h) include/nccl.h

all: lib oracle numerics-host bootstrap-test tuner-test nccl-perf comm-examples plan-test mapcheck-test xgmi-probe atomicity-probe \
     fp8-probe release-probe reuse-probe export-check-test barrier-probe

.PHONY: export-check-test
export-check-test: tests/native/export_check_test

lib: $(LIBDIR)/libnccl.so

$(BUILD)/%.o: $(SRCDIR)/%.cc $(HDRS)
	@mkdir -p $(BUILD)
	$(CXX) $(COMMON) -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c $< -o $@

# The kernels' register / scratch / occupancy report goes to build/<name>.usage
# (tests/test_occupancy.py checks that every channel kernel fits two workgroups per CU).
$(BUILD)/%.o: $(SRCDIR)/%.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -Rpass-analysis=kernel-resource-usage -c $< -o $@ 2> $(BUILD)/$*.usage; \
	  st=$$?; grep -E "warning|error" $(BUILD)/$*.usage >&2; exit $$st

# -Wl,--version-script: export exactly nccl* / pnccl* (reference src/libnccl.map:13-19)
$(LIBDIR)/libnccl.so: $(HOSTOBJ) $(DEVOBJ) $(SRCDIR)/libnccl.map
	@mkdir -p $(LIBDIR)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -Wl,-soname,libnccl.so.2 -Wl,-Bsymbolic \
	  -Wl,--version-script=$(SRCDIR)/libnccl.map -o $@ $(HOSTOBJ) $(DEVOBJ) -lpthread -ldl
	ln -sf libnccl.so $(LIBDIR)/libnccl.so.2

oracle: oracle/_build/liboracle.so

oracle/_build/liboracle.so: oracle/nccl_oracle.c
	@mkdir -p oracle/_build
	gcc -O2 -fPIC -shared -fopenmp -ffp-contract=off -fno-fast-math -std=c11 -o $@ $< -lm

clean:
	rm -rf $(BUILD) $(LIBDIR) oracle/_build

.PHONY: all lib oracle clean

# test-only host build of the kernels' numerics, checked exhaustively against the oracle
numerics-host: build/libnumerics_host.so

build/libnumerics_host.so: tests/native/numerics_host.cc $(SRCDIR)/numerics.h
	@mkdir -p build
	$(CXX) -O2 -std=c++17 -fPIC -shared -ffp-contract=off -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -o $@ $<

.PHONY: numerics-host

# test-only host program exercising the TCP bootstrap across forked processes
bootstrap-test: build/bootstrap_test

build/bootstrap_test: tests/native/bootstrap_test.cc $(SRCDIR)/bootstrap.cc $(SRCDIR)/debug.cc $(HDRS)
	@mkdir -p build
	$(CXX) -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -o $@ tests/native/bootstrap_test.cc \
	  $(SRCDIR)/bootstrap.cc $(SRCDIR)/debug.cc -lpthread

.PHONY: bootstrap-test

# test-only tuner plugin (reference ABI v6) loaded through NCCL_TUNER_PLUGIN by the GPU tests
tuner-test: tests/native/libnccl-tuner-test.so

tests/native/libnccl-tuner-test.so: tests/native/tuner_plugin.c include/nccl_tuner.h include/nccl.h
	gcc -O2 -fPIC -shared -fvisibility=hidden -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -o $@ $<

.PHONY: tuner-test

# nccl-tests-style native driver written against include/nccl.h only (C ABI check + Python-free timing)
nccl-perf: tests/native/nccl_perf

tests/native/nccl_perf: tests/native/nccl_perf.cc include/nccl.h $(LIBDIR)/libnccl.so
	$(HIPCC) -O2 --offload-arch=$(ARCH) -Iinclude -o $@ $< -L$(LIBDIR) -lnccl -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'

.PHONY: nccl-perf

# the reference's communicator-creation examples (pthread per rank, ncclCommInitAll) + a known-answer AllReduce
comm-examples: tests/native/comm_examples

tests/native/comm_examples: tests/native/comm_examples.cc include/nccl.h $(LIBDIR)/libnccl.so
	$(HIPCC) -O2 --offload-arch=$(ARCH) -Iinclude -o $@ $< -L$(LIBDIR) -lnccl -lpthread -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'

.PHONY: comm-examples

# CU-driven peer bandwidth probe (run by bench.py's suite on multi-GPU nodes)
xgmi-probe: tests/native/xgmi_probe

tests/native/xgmi_probe: tests/native/xgmi_probe.hip
	$(HIPCC) -O2 --offload-arch=$(ARCH) -o $@ $<

.PHONY: xgmi-probe

# CPU test driver of enqueue.cc's planning (no GPU: launches and the few HIP calls are stubbed)
plan-test: tests/native/plan_test

tests/native/plan_test: tests/native/plan_test.cc $(SRCDIR)/enqueue.cc $(SRCDIR)/debug.cc $(HDRS)
	$(CXX) -O1 -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -o $@ tests/native/plan_test.cc \
	  $(SRCDIR)/enqueue.cc $(SRCDIR)/debug.cc -lpthread

.PHONY: plan-test

# Host sanitizer builds (SURVEY §5 race detection; tests/test_sanitizers.py): the bootstrap, the IPC fd server
# and the planning code under ASan+UBSan and, separately, TSan. Host code only — no GPU code is instrumented.
SANCXX   := $(CXX) -g -O1 -fno-omit-frame-pointer -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude
ASAN     := -fsanitize=address,undefined -fno-sanitize-recover=undefined
TSAN     := -fsanitize=thread
HIPRT    := -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
SANBIN   := build/asan/bootstrap_test build/asan/plan_test build/asan/ipc_server_test \
            build/tsan/bootstrap_test build/tsan/ipc_server_test
sanitize: $(SANBIN)

build/asan/bootstrap_test build/tsan/bootstrap_test: tests/native/bootstrap_test.cc $(SRCDIR)/bootstrap.cc $(SRCDIR)/debug.cc $(HDRS)
	@mkdir -p $(dir $@)
	$(SANCXX) $(if $(findstring asan,$@),$(ASAN),$(TSAN)) -o $@ tests/native/bootstrap_test.cc $(SRCDIR)/bootstrap.cc \
	  $(SRCDIR)/debug.cc -lpthread

build/asan/ipc_server_test build/tsan/ipc_server_test: tests/native/ipc_server_test.cc $(SRCDIR)/ipc.cc $(SRCDIR)/debug.cc $(HDRS)
	@mkdir -p $(dir $@)
	$(SANCXX) $(if $(findstring asan,$@),$(ASAN),$(TSAN)) -o $@ tests/native/ipc_server_test.cc $(SRCDIR)/ipc.cc \
	  $(SRCDIR)/debug.cc -lpthread $(HIPRT)

# CPU test of the stale dma-buf export checks (ipc.cc ipcAdmitExport) with memfd files in place of dma-bufs
tests/native/export_check_test: tests/native/export_check_test.cc $(SRCDIR)/ipc.cc $(SRCDIR)/debug.cc $(HDRS)
	$(CXX) -O1 -g -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -o $@ tests/native/export_check_test.cc \
	  $(SRCDIR)/ipc.cc $(SRCDIR)/debug.cc -lpthread $(HIPRT)

build/asan/plan_test: tests/native/plan_test.cc $(SRCDIR)/enqueue.cc $(SRCDIR)/debug.cc $(HDRS)
	@mkdir -p $(dir $@)
	$(SANCXX) $(ASAN) -o $@ tests/native/plan_test.cc $(SRCDIR)/enqueue.cc $(SRCDIR)/debug.cc -lpthread

.PHONY: sanitize

# store-atomicity probe (torn 8/16/64/128-byte lines under concurrent write-through stores; GPU test + bench suite)
atomicity-probe: tests/native/store_atomicity_probe

tests/native/store_atomicity_probe: tests/native/store_atomicity_probe.hip
	$(HIPCC) -O3 --offload-arch=$(ARCH) -o $@ $<

.PHONY: atomicity-probe

# fp8 conversion probe: gfx950's fp8 convert instructions vs numerics.h's software conversions, every code and
# every half value (GPU test tests/test_gpu_numerics.py; decides the hardware fp8 path)
fp8-probe: tests/native/fp8_cvt_probe tests/native/fp8_f16_probe

tests/native/fp8_f16_probe: tests/native/fp8_f16_probe.hip $(SRCDIR)/numerics.h
	$(HIPCC) -O3 --offload-arch=$(ARCH) -ffp-contract=off -fno-gpu-flush-denormals-to-zero -o $@ $<

tests/native/fp8_cvt_probe: tests/native/fp8_cvt_probe.hip $(SRCDIR)/numerics.h
	$(HIPCC) -O3 --offload-arch=$(ARCH) -ffp-contract=off -fno-gpu-flush-denormals-to-zero -o $@ $<

.PHONY: fp8-probe

# CPU test driver of the init-time mapping check (mapcheck.cc) with the device and the imports stubbed
mapcheck-test: tests/native/mapcheck_test

tests/native/mapcheck_test: tests/native/mapcheck_test.cc $(SRCDIR)/mapcheck.cc $(SRCDIR)/debug.cc $(HDRS)
	$(CXX) -O1 -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -o $@ tests/native/mapcheck_test.cc \
	  $(SRCDIR)/mapcheck.cc $(SRCDIR)/debug.cc -lpthread

.PHONY: mapcheck-test

# does a kernel queued behind another on the same stream start while the first is resident?
barrier-probe: tests/native/barrier_probe

tests/native/barrier_probe: tests/native/barrier_probe.hip
	$(HIPCC) -O2 --offload-arch=$(ARCH) -o $@ $<

.PHONY: barrier-probe

# does unmapping an imported dma-buf mapping wait for the device? (decides where peers' mappings are released,
# DESIGN.md §3.2)
release-probe: tests/native/release_probe

tests/native/release_probe: tests/native/release_probe.hip
	$(HIPCC) -O2 --offload-arch=$(ARCH) -o $@ $<

.PHONY: release-probe

# the importer's unmap-then-allocate pattern of eager registration churn, without the library
reuse-probe: tests/native/reuse_probe

tests/native/reuse_probe: tests/native/reuse_probe.hip
	$(HIPCC) -O2 --offload-arch=$(ARCH) -o $@ $<

.PHONY: reuse-probe
