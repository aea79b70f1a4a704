# Build recipe for the MI355X bling core.  `python -c "import __graft_entry__ as g; g.build()"` runs
# `make -j8 all`.  Outputs stay in-tree (git-ignored, but they travel to the GPU box with gpurun).
#
#   bling_amd/_lib/libbling_host.so   host: .bling loader + film output   (g++)
#   bling_amd/_lib/libbling_hip.so    device core: BVH, kernels, C ABI    (hipcc, gfx950)
#   oracle/_build/liboracle.so        CPU oracle (test infrastructure)     (g++ + OpenMP)
#   bling_amd/_lib/bling              C++ command-line renderer (host front end)
#   bling_amd/_lib/libbling_mathcheck.so  exhaustive device check of common/fast_cr.h (tests)

HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
ARCH     ?= gfx950
LIBDIR   := bling_amd/_lib
ORADIR   := oracle/_build
space    := $(subst ,, )

HOST_SRC := bling_amd/csrc/host/loader.cpp
HOST_HDR := bling_amd/csrc/host/hmath.h bling_amd/csrc/common/sky_model.h bling_amd/csrc/common/scene_features.h \
            bling_amd/csrc/common/spectral_data.h bling_amd/csrc/common/perlin.h include/bling_scene.h include/bling_host.h \
            bling_amd/csrc/common/image_tex.h bling_amd/csrc/common/cr_math.h bling_amd/csrc/host/image_io.h
CORE_SRC := $(wildcard bling_amd/csrc/core/*.hip) $(wildcard bling_amd/csrc/core/*.cpp)
# STUB (experiment builds only) is part of the object directory: stubbed units never mix with real ones
ifneq ($(strip $(STUB)),)
ifeq ($(strip $(V)),)
$(error STUB is for experiment builds only: give it a variant name, make variant V=name STUB="4 5")
endif
endif
OBJDIR   := build/core$(if $(V),_$(V),)$(if $(strip $(STUB)),_stub$(subst $(space),,$(strip $(STUB))),)
CORE_OBJ := $(patsubst bling_amd/csrc/core/%,$(OBJDIR)/%.o,$(CORE_SRC))
CORE_HDR := $(wildcard bling_amd/csrc/core/*.h) bling_amd/csrc/common/sky_model.h \
            bling_amd/csrc/common/spectral_data.h bling_amd/csrc/common/counter_rng.h include/bling.h include/bling_scene.h \
            bling_amd/csrc/common/scene_features.h bling_amd/csrc/common/perlin.h bling_amd/csrc/common/cr_math.h \
            bling_amd/csrc/common/fast_cr.h bling_amd/csrc/common/cellnoise.h bling_amd/csrc/common/image_tex.h
ORA_SRC  := $(wildcard oracle/*.cpp)
ORA_HDR  := $(wildcard oracle/*.h) include/bling_scene.h bling_amd/csrc/common/perlin.h bling_amd/csrc/common/cr_math.h \
            bling_amd/csrc/common/cellnoise.h bling_amd/csrc/common/image_tex.h

# GHC emits no fused multiply-adds: the oracle and the loader keep every binary32 rounding.
HOSTFLAGS := -O2 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function
HIPFLAGS  := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -fno-gpu-rdc \
             -Wno-unused-result -munsafe-fp-atomics

all: $(LIBDIR)/libbling_host.so $(LIBDIR)/libbling_hip.so $(ORADIR)/liboracle.so $(LIBDIR)/bling \
     $(LIBDIR)/libbling_mathcheck.so

host: $(LIBDIR)/libbling_host.so
oracle: $(ORADIR)/liboracle.so
core: $(LIBDIR)/libbling_hip.so

$(LIBDIR)/libbling_host.so: $(HOST_SRC) $(HOST_HDR)
	@mkdir -p $(LIBDIR)
	$(CXX) $(HOSTFLAGS) -shared -o $@ $(HOST_SRC) -lz

$(ORADIR)/liboracle.so: $(ORA_SRC) $(ORA_HDR)
	@mkdir -p $(ORADIR)
	$(CXX) $(HOSTFLAGS) -fopenmp -shared -o $@ $(ORA_SRC)

# one object per unit (core, sppm driver, one per kernel feature profile) so make -j compiles the
# kernel instantiations in parallel
$(OBJDIR)/%.o: bling_amd/csrc/core/% $(CORE_HDR)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(DEFS) $(STUBDEF) -c -o $@ $<

$(LIBDIR)/libbling_hip.so: $(CORE_OBJ)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(CORE_OBJ)

$(LIBDIR)/bling: bling_amd/csrc/host/bling_main.cpp $(LIBDIR)/libbling_host.so $(LIBDIR)/libbling_hip.so
	$(CXX) -O2 -std=c++17 -o $@ bling_amd/csrc/host/bling_main.cpp -I include \
	   -L$(LIBDIR) -lbling_host -lbling_hip -Wl,-rpath,'$$ORIGIN'

$(LIBDIR)/libbling_mathcheck.so: bling_amd/csrc/check/mathcheck.hip bling_amd/csrc/common/fast_cr.h bling_amd/csrc/common/cr_math.h
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<

# experiment builds: make variant V=name DEFS="-DBLING_SHADE_WAVES=4" -> libbling_hip_name.so,
# selected at run time with BLING_HIP_VARIANT=name.  STUB="4 5" stubs those profile units (their
# entry points throw) to cut the build time of an A/B of the bench configs.
$(foreach k,$(STUB),$(foreach u,$(filter $(OBJDIR)/prof_$(k).hip.o $(OBJDIR)/prof_$(k)a.hip.o $(OBJDIR)/prof_$(k)b.hip.o $(OBJDIR)/prof_$(k)c.hip.o,$(CORE_OBJ)),$(eval $(u): STUBDEF := -DBLING_STUB_PROFILE)))
variant: $(CORE_OBJ)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $(LIBDIR)/libbling_hip_$(V).so $(CORE_OBJ)

clean:
	rm -rf $(LIBDIR) $(ORADIR) build

.PHONY: all host oracle core clean variant
