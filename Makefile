# Build of the MI355X rasterizer library and the CPU oracle (test infrastructure).
#   make          -> gaussiansplatting_amd/lib/libgs_mi355x.so, oracle/libgs_oracle.so
#   make -j16     (gpurun boxes: at most -j16)
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
LIBDIR  := gaussiansplatting_amd/lib
OBJDIR  := build/obj
SRC     := gaussiansplatting_amd/csrc
# -fno-slp-vectorize: packed f32 VALU ops (v_pk_*_f32) issue at half rate on gfx950 (measured,
# scripts/valu_probe.hip), so SLP packing of scalar code buys nothing and adds register moves.
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
            -fno-slp-vectorize -Wall -Wno-unused-function -Wno-unused-result
HDRS    := $(wildcard $(SRC)/*.hpp) include/gs_rasterizer.h
OBJS    := $(OBJDIR)/gs_sort.o $(OBJDIR)/gs_segsort.o $(OBJDIR)/gs_raster.o $(OBJDIR)/gs_blend.o $(OBJDIR)/gs_chain.o $(OBJDIR)/gs_density.o $(OBJDIR)/gs_optim.o $(OBJDIR)/gs_loss.o $(OBJDIR)/gs_membw.o $(OBJDIR)/gs_io.o $(OBJDIR)/gs_capi.o

all: $(LIBDIR)/libgs_mi355x.so oracle/libgs_oracle.so $(LIBDIR)/gs_train_headless

$(OBJDIR)/%.o: $(SRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/gs_capi.o: $(SRC)/gs_capi.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

# host-only C++ (scene formats): no device code
$(OBJDIR)/gs_io.o: $(SRC)/gs_io.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) -O2 -std=c++17 -fPIC -ffp-contract=off -Wall -c $< -o $@

$(LIBDIR)/libgs_mi355x.so: $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

$(LIBDIR)/gs_train_headless: $(SRC)/gs_train_headless.cpp include/gs_tiled_rasterizer.hpp $(LIBDIR)/libgs_mi355x.so
	$(HIPCC) -O2 -std=c++17 -Wno-unused-result -Wno-unused-value -o $@ $< -L$(LIBDIR) -lgs_mi355x -Wl,-rpath,'$$ORIGIN'

oracle/libgs_oracle.so: oracle/gs_oracle.c oracle/gs_oracle.h include/gs_rasterizer.h
	gcc -O3 -march=x86-64-v3 -std=c11 -fPIC -shared -fopenmp -ffp-contract=off -fno-fast-math \
	    -Wall -o $@ oracle/gs_oracle.c -lm

# AddressSanitizer + UndefinedBehaviorSanitizer build of the host code that parses untrusted files
# (gs_io.cpp) and of the CPU oracle, driven by tests/sanitize/san_main.cpp (tests/test_sanitize.py)
SANFLAGS := -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
            -ffp-contract=off -fno-fast-math
sanitize: build/san/gs_san

build/san/gs_san: tests/sanitize/san_main.cpp tests/sanitize/io_shim.cpp $(SRC)/gs_io.cpp oracle/gs_oracle.c oracle/gs_oracle.h include/gs_rasterizer.h
	@mkdir -p build/san
	gcc $(SANFLAGS) -std=c11 -fopenmp -Wall -Iinclude -c oracle/gs_oracle.c -o build/san/gs_oracle.o
	g++ $(SANFLAGS) -std=c++17 -Wall -Iinclude -Ioracle tests/sanitize/san_main.cpp tests/sanitize/io_shim.cpp \
	    $(SRC)/gs_io.cpp build/san/gs_oracle.o -fopenmp -lm -o $@

clean:
	rm -rf $(OBJDIR) build/san $(LIBDIR)/libgs_mi355x.so $(LIBDIR)/gs_train_headless oracle/libgs_oracle.so

.PHONY: all clean sanitize
