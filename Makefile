# Builds libleastereo_hip.so for gfx950 (MI355X) in-tree, plus the oracle's
# nothing-to-build marker.  `make -j8` here; the GPU box uses the prebuilt .so.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall -Wno-unused-function \
            -Iinclude -Ileastereo_amd/csrc -munsafe-fp-atomics
SRC      := $(wildcard leastereo_amd/csrc/*.hip)
OBJ      := $(patsubst leastereo_amd/csrc/%.hip,build/obj/%.o,$(SRC))
LIB      := leastereo_amd/libleastereo_hip.so

all: $(LIB)

# the Winograd engines: SLP-packed f32 VALU (v_pk_*) beside MFMAs costs more issue
# cycles than the scalar pairs it replaces (MI355X_MICROARCH.md, filler prices)
build/obj/conv3d_wino.o build/obj/conv3d_wino2.o build/obj/conv3d_wino44.o: HIPFLAGS += -fno-slp-vectorize

build/obj/%.o: leastereo_amd/csrc/%.hip $(wildcard leastereo_amd/csrc/*.h) include/leastereo_hip.h include/leastereo_hip_tuning.h
	@mkdir -p build/obj
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJ)

resource-usage: $(SRC)
	@mkdir -p build/ru
	for f in $(SRC); do $(HIPCC) $(HIPFLAGS) -c $$f -o build/ru/$$(basename $$f).o -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size" ; done

# Host-side AddressSanitizer build of the C-ABI boundary: every unit with
# ASan on its host side only (the device code is built as usual and never launched:
# the driver, tests/asan/capi_asan.cpp, drives each entry point through its argument
# checks and the host queries).  Runs on a machine without a GPU.
ASANFLAGS := -O1 -g -std=c++17 -fPIC --offload-arch=$(ARCH) -Iinclude -Ileastereo_amd/csrc -Xarch_host -fsanitize=address \
             -Xarch_host -fno-omit-frame-pointer
ASANOBJ   := $(patsubst leastereo_amd/csrc/%.hip,build/asan/%.o,$(SRC))

build/asan/%.o: leastereo_amd/csrc/%.hip $(wildcard leastereo_amd/csrc/*.h) include/leastereo_hip.h include/leastereo_hip_tuning.h
	@mkdir -p build/asan
	$(HIPCC) $(ASANFLAGS) -c $< -o $@

build/asan/capi_asan_main.o: tests/asan/capi_asan.cpp include/leastereo_hip.h include/leastereo_hip_tuning.h
	@mkdir -p build/asan
	$(HIPCC) $(ASANFLAGS) -c $< -o $@

build/asan/capi_asan: build/asan/capi_asan_main.o $(ASANOBJ)
	$(HIPCC) --offload-arch=$(ARCH) -fno-gpu-sanitize -fsanitize=address -o $@ $^

asan: build/asan/capi_asan
	ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 ./build/asan/capi_asan

clean:
	rm -rf build $(LIB)

.PHONY: all clean resource-usage asan
