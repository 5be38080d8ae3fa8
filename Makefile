# Build of the MI355X BPE library (gfx950).  `make` builds:
#   llmtokenizer_amd/libbpe_amd.so  C-ABI: include/bpe.h, bpe_ex.h, bpe_gpu.h
#   tools/bpe_main                  reference-compatible CLI
#   oracle/                         CPU checker (test infrastructure only)
HIPCC ?= /opt/rocm/bin/hipcc
CC ?= gcc
ARCH ?= gfx950
JOBS ?= 8
PKG := llmtokenizer_amd
BUILD := $(PKG)/build
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wno-unused-result -Wno-unused-value
CFLAGS := -O2 -g -fPIC -Wall -Wextra -Wno-unused-parameter -std=c11 -D_GNU_SOURCE

CSRC := $(PKG)/src/bpe.c $(PKG)/src/dyn_arr.c $(PKG)/src/hash_table.c
COBJ := $(patsubst $(PKG)/src/%.c,$(BUILD)/%.o,$(CSRC))
HIPDEPS := $(wildcard $(PKG)/csrc/*.hip $(PKG)/csrc/*.h) include/bpe_gpu.h

all: $(PKG)/libbpe_amd.so tools/bpe_main oracle

$(BUILD):
	mkdir -p $(BUILD)

$(BUILD)/engine.o: $(HIPDEPS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $(PKG)/csrc/engine.hip -o $@

$(BUILD)/%.o: $(PKG)/src/%.c $(wildcard include/*.h) | $(BUILD)
	$(CC) $(CFLAGS) -c $< -o $@

$(PKG)/libbpe_amd.so: $(BUILD)/engine.o $(COBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -lm -ldl -lpthread

tools/bpe_main: tools/bpe_main.c $(PKG)/libbpe_amd.so
	$(CC) -O2 -Iinclude -o $@ $< -L$(PKG) -lbpe_amd -Wl,-rpath,'$$ORIGIN/../$(PKG)'

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD) $(PKG)/libbpe_amd.so tools/bpe_main
	$(MAKE) -C oracle clean

.PHONY: all oracle clean

# Host C library under AddressSanitizer + UBSan (device calls stubbed:
# tests/asan/gpu_stub.c); run by tests/test_asan_host.py
tests/asan/asan_host: tests/asan/asan_host.c tests/asan/gpu_stub.c $(CSRC) $(wildcard include/*.h)
	$(CC) -O1 -g -std=c11 -D_GNU_SOURCE -fno-omit-frame-pointer -fsanitize=address,undefined \
	    -fno-sanitize-recover=undefined -Iinclude -o $@ tests/asan/asan_host.c tests/asan/gpu_stub.c $(CSRC) -lm -lpthread

asan-host: tests/asan/asan_host
.PHONY: asan-host
