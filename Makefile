# mpx — MI355X-native build (gfx950 only; hipcc cross-compiles without a GPU).
#
#   make            libmpx (.so for Python, .a for the CLIs) + every program
#   make lib        cuda_mpi_openmp_amd/_lib/libmpx.so only
#   make clean
#
# Program layout keeps the reference harness contract: the lab is derived from
# the grandparent directory of the binary (reference run_test.py:58-60), so the
# lab programs live in labs/labN/src/.

ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
CC        ?= gcc
ARCH      ?= gfx950

INC       := -Inative/include -I$(ROCM)/include
# warnings are errors (-Wall -Werror); make WERROR= to relax
WERROR    ?= -Werror
HIPFLAGS  := --offload-arch=$(ARCH) -mcode-object-version=5 -O3 -std=c++17 -fPIC \
             -ffp-contract=off -Wall -Wno-unused-function $(WERROR) $(INC)
COPT      := -O3 -fopenmp -ffp-contract=off -fPIC -Wall $(WERROR) -std=gnu11 -Inative/include
CSER      := -O0 -ffp-contract=off -Wall -Wno-unknown-pragmas $(WERROR) -std=gnu11 -Inative/include

B         := build
PYLIB     := cuda_mpi_openmp_amd/_lib/libmpx.so
TUNELIB   := cuda_mpi_openmp_amd/_lib/libmpx_tune.so
ALIB      := $(B)/libmpx.a

HIP_SRCS  := $(wildcard native/src/kernels/*.hip)
HIP_OBJS  := $(patsubst native/src/kernels/%.hip,$(B)/k_%.o,$(HIP_SRCS))
CORE_OBJS := $(B)/capi.o $(B)/comm.o $(B)/ipc.o
CPU_OBJ   := $(B)/cpu_kernels.o
LIB_OBJS  := $(HIP_OBJS) $(CORE_OBJS) $(CPU_OBJ)
HDRS      := $(wildcard native/include/mpx/*.h native/include/mpx/*.hpp native/src/kernels/*.hpp native/src/cpu/*.h)

LABS      := labs/lab1/src labs/lab2/src labs/lab3/src labs/lab5/src
GPU_APPS  := $(foreach L,1 2 3 5,labs/lab$(L)/src/to_plot_hip_exe labs/lab$(L)/src/hip_exe)
CPU_APPS  := $(foreach L,1 2 3 5,labs/lab$(L)/src/cpu_exe labs/lab$(L)/src/cpu_omp_exe)
MISC_APPS := labs/lab3/src/read_input_exe bin/gpu_info bin/hw1 bin/hw2 bin/mpx_mgpu

.PHONY: all lib apps tools tune clean
all: lib apps tune
lib: $(PYLIB) $(ALIB)
# tuning-only kernel variants / probes (tools/kbench.py), linked against libmpx
tune: $(TUNELIB)
apps: $(GPU_APPS) $(CPU_APPS) $(MISC_APPS)

$(B):
	@mkdir -p $(B) bin cuda_mpi_openmp_amd/_lib

$(LABS):
	@mkdir -p $@

$(B)/k_%.o: native/src/kernels/%.hip $(HDRS) | $(B)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# the lab2 kernels keep scalar v_fmac chains: SLP packing into v_pk_fma_f32 costs
# hazard NOPs and ~40 VGPRs (8 -> 4 waves per SIMD) for no extra FLOP rate
$(B)/k_edge.o $(B)/k_edge_roberts.o $(B)/k_edge_stream.o $(B)/t_edge_variants.o: HIPFLAGS += -fno-slp-vectorize
# MFMA accumulators straight into VGPRs (unified file on gfx950): no v_accvgpr_read per result
$(B)/k_classify.o: HIPFLAGS += -mllvm -amdgpu-mfma-vgpr-form

$(B)/capi.o: native/src/core/capi.cpp $(HDRS) | $(B)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(B)/ipc.o: native/src/core/ipc.cpp $(HDRS) | $(B)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# RCCL is not linked: comm.cpp binds the librccl torch already loaded (dlsym)
$(B)/comm.o: native/src/core/comm.cpp $(HDRS) | $(B)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(B)/cpu_kernels.o: native/src/cpu/cpu_kernels.c $(HDRS) | $(LABS)
	$(CC) $(COPT) -c $< -o $@

$(PYLIB): $(LIB_OBJS) | $(B)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(LIB_OBJS) -lgomp -lm -ldl

$(B)/t_%.o: native/tune/%.hip $(HDRS) | $(B)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

TUNEOBJ   := $(B)/t_edge_variants.o $(B)/t_sort_variants.o $(B)/t_jacobi_variants.o $(B)/t_vsub_variants.o
$(TUNELIB): $(TUNEOBJ) $(PYLIB)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(TUNEOBJ) -L$(dir $(PYLIB)) -lmpx -Wl,-rpath,'$$ORIGIN'

$(ALIB): $(LIB_OBJS) | $(B)
	rm -f $@ && ar rcs $@ $(LIB_OBJS)

# ---- GPU programs: two personalities from one source ----
# linked against libmpx.so (one copy of the kernels on disk, not one per
# program); found through the build tree's absolute path (tests copy a lab to
# a scratch directory) and, relocated, next to the repository layout
LIBDIR    := $(abspath $(dir $(PYLIB)))
SOLINK    := -L$(LIBDIR) -lmpx -Wl,-rpath,$(LIBDIR)
labs/lab%/src/to_plot_hip_exe: native/apps/lab%_gpu.cpp $(PYLIB) $(HDRS) | $(LABS)
	$(HIPCC) $(HIPFLAGS) $< $(SOLINK) -Wl,-rpath,'$$ORIGIN/../../../cuda_mpi_openmp_amd/_lib' -lgomp -lm -ldl -o $@

labs/lab%/src/hip_exe: native/apps/lab%_gpu.cpp $(PYLIB) $(HDRS) | $(LABS)
	$(HIPCC) $(HIPFLAGS) -DMPX_SUBMISSION $< $(SOLINK) -Wl,-rpath,'$$ORIGIN/../../../cuda_mpi_openmp_amd/_lib' -lgomp -lm -ldl -o $@

# ---- CPU references: serial -O0 (published methodology) and OpenMP -O3 ----
labs/lab%/src/cpu_exe: native/apps/lab%_cpu.c native/src/cpu/cpu_kernels.c $(HDRS) | $(LABS)
	$(CC) $(CSER) $< native/src/cpu/cpu_kernels.c -lm -o $@

labs/lab%/src/cpu_omp_exe: native/apps/lab%_cpu.c native/src/cpu/cpu_kernels.c $(HDRS) | $(LABS)
	$(CC) $(COPT) $< native/src/cpu/cpu_kernels.c -lm -o $@

labs/lab3/src/read_input_exe: native/apps/lab3_read_input.c | $(LABS)
	$(CC) $(CSER) $< -o $@

bin/gpu_info: native/apps/gpu_info.cpp $(PYLIB) $(HDRS) | $(B)
	$(HIPCC) $(HIPFLAGS) $< $(SOLINK) -Wl,-rpath,'$$ORIGIN/../cuda_mpi_openmp_amd/_lib' -lgomp -lm -ldl -o $@

# native multi-GPU runtime: links /opt/rocm's RCCL directly (no torch in this process)
bin/mpx_mgpu: native/apps/mpx_mgpu.cpp $(PYLIB) $(HDRS) | $(B)
	$(HIPCC) $(HIPFLAGS) $< $(SOLINK) -Wl,-rpath,'$$ORIGIN/../cuda_mpi_openmp_amd/_lib' -L$(ROCM)/lib -lrccl -lgomp -lm -ldl -lpthread -Wl,-rpath,$(ROCM)/lib -o $@

bin/hw1: native/apps/hw1_quadratic.c | $(B)
	$(CC) $(CSER) $< -lm -o $@

bin/hw2: native/apps/hw2_bubble_sort.c | $(B)
	$(CC) $(CSER) $< -o $@

# ---- stand-alone measurement tools (not part of `all`) ----
tools: bin/mfma_valu_overlap
bin/mfma_valu_overlap: tools/experiments/mfma_valu_overlap.hip | $(B)
	$(HIPCC) --offload-arch=$(ARCH) -O3 $< -o $@

# ---- host-only sanitizer builds of the CPU references ----
# GPU ASan / xnack+ code objects are not available on the MI355X pool, so the
# sanitizers cover the host code paths: the CPU references, the .data / text
# I/O and the stdin parsers shared with the GPU programs.
SAN       := -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all
SAN_APPS  := $(foreach L,1 2 3 5,build/san/lab$(L)_cpu_exe build/san/lab$(L)_cpu_omp_exe) build/san/lab3_read_input_exe \
             build/san/hw1 build/san/hw2
.PHONY: sanitize
sanitize: $(SAN_APPS)

build/san:
	@mkdir -p build/san

build/san/lab%_cpu_exe: native/apps/lab%_cpu.c native/src/cpu/cpu_kernels.c $(HDRS) | build/san
	$(CC) $(SAN) -ffp-contract=off -Wall -Wno-unknown-pragmas -std=gnu11 -Inative/include $< native/src/cpu/cpu_kernels.c -lm -o $@

build/san/lab%_cpu_omp_exe: native/apps/lab%_cpu.c native/src/cpu/cpu_kernels.c $(HDRS) | build/san
	$(CC) $(SAN) -fopenmp -ffp-contract=off -Wall -std=gnu11 -Inative/include $< native/src/cpu/cpu_kernels.c -lm -o $@

build/san/lab3_read_input_exe: native/apps/lab3_read_input.c | build/san
	$(CC) $(SAN) -Wall -std=gnu11 $< -o $@

build/san/hw1: native/apps/hw1_quadratic.c | build/san
	$(CC) $(SAN) -Wall -std=gnu11 $< -lm -o $@

build/san/hw2: native/apps/hw2_bubble_sort.c | build/san
	$(CC) $(SAN) -Wall -std=gnu11 $< -o $@

clean:
	rm -rf $(B) bin $(PYLIB) $(TUNELIB) $(GPU_APPS) $(CPU_APPS) labs/lab3/src/read_input_exe
