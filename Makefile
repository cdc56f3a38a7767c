# Builds libgrk.so (HIP kernels + C ABI) for gfx950, in-tree, and the C oracle.
#   make            -> tencent_recommendation_2025_amd/libgrk.so
#   make -j8 ...    (object files go to build/)
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
SRC_DIR := tencent_recommendation_2025_amd/csrc
OBJ_DIR := build/obj
LIB     := tencent_recommendation_2025_amd/libgrk.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Iinclude -Wall -Wno-unused-function \
            -Wno-unused-variable -Wno-unused-but-set-variable
HIP_SRCS := $(wildcard $(SRC_DIR)/*.hip)
CPP_SRCS := $(wildcard $(SRC_DIR)/*.cpp)
OBJS := $(patsubst $(SRC_DIR)/%.hip,$(OBJ_DIR)/%.o,$(HIP_SRCS)) $(patsubst $(SRC_DIR)/%.cpp,$(OBJ_DIR)/%.cpp.o,$(CPP_SRCS))

all: $(LIB)

# whole-sequence attention: MFMA accumulators in VGPRs (no AGPR<->VGPR copies
# around the S tile).  Every S/dP chain starts from acc_zero() (grk_mfma.h):
# with a literal zero srcC this form let an MFMA's vdst alias its own srcA/srcB,
# which gave timing-dependent wrong HSTU rows when two workgroups shared a CU
# (DESIGN.md §5b); the overlap check below guards the link.
$(OBJ_DIR)/grk_attention_seq.o: HIPFLAGS += -mllvm -amdgpu-mfma-vgpr-form
# no SLP packing of the scalar score math into v_pk_*_f32: packed f32 VALU is
# slower than scalar beside MFMAs, and packed SiLU chains in the forward gave
# run-to-run different outputs
$(OBJ_DIR)/grk_attention_seq.o: HIPFLAGS += -fno-slp-vectorize

# residual quantisation: codes must be a pure function of fp32 inputs (no FMA
# contraction of the squared differences; oracle/rqvae.py restates the order)
$(OBJ_DIR)/grk_rqvae.o: HIPFLAGS += -ffp-contract=off

$(OBJ_DIR):
	mkdir -p $@

$(OBJ_DIR)/%.o: $(SRC_DIR)/%.hip $(wildcard $(SRC_DIR)/*.h) include/grk.h | $(OBJ_DIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(OBJ_DIR)/%.cpp.o: $(SRC_DIR)/%.cpp include/grk.h | $(OBJ_DIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

HIP_OBJS := $(patsubst $(SRC_DIR)/%.hip,$(OBJ_DIR)/%.o,$(HIP_SRCS))

# no MFMA may write registers it reads as srcA/srcB (scripts/check_mfma_overlap.py)
$(LIB): $(OBJS)
	python3 scripts/check_mfma_overlap.py $(HIP_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -L/opt/rocm/lib -lhipblaslt

clean:
	rm -rf build $(LIB)

.PHONY: all clean
