# Build libcairo_amd.so (HIP for gfx950 + host C++) and the test oracle.
# `python -c "import __graft_entry__ as g; g.build()"` runs this.
HIPCC   ?= /opt/rocm/bin/hipcc
CXX     = g++
ARCH    ?= gfx950
CXXFLAGS = -O3 -std=c++17 -fPIC -pthread -Wall -Wno-unused-function
HIPFLAGS = --offload-arch=$(ARCH) $(CXXFLAGS) -munsafe-fp-atomics
SRC      = cairo_amd/csrc
OBJ      = build/obj
LIB      = cairo_amd/_lib/libcairo_amd.so
ORACLE   = oracle/liboracle.so
API_BIN  = cairo_amd/_lib/evx1_api_caller

HIP_SRCS = $(SRC)/kernels.hip $(SRC)/backend.hip $(SRC)/precode.hip
CPP_SRCS = $(SRC)/entropy.cpp $(SRC)/bitstream.cpp $(SRC)/encoder.cpp $(SRC)/decoder.cpp $(SRC)/pipeline.cpp $(SRC)/unserialize.cpp
OBJS     = $(patsubst $(SRC)/%.hip,$(OBJ)/%.o,$(HIP_SRCS)) $(patsubst $(SRC)/%.cpp,$(OBJ)/%.o,$(CPP_SRCS))
HDRS     = $(wildcard $(SRC)/*.h) $(wildcard include/*.h)

HOP_BIN  = tools/bin/hop_latency

all: $(LIB) $(ORACLE) $(API_BIN) $(HOP_BIN)

# Hand-off latency micro-benchmark: one hop of the progress-word
# protocol between two workgroups, in one process or across two.
$(HOP_BIN): tools/hop_latency.hip
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

$(OBJ)/%.o: $(SRC)/%.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/%.o: $(SRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJ)
	$(CXX) $(CXXFLAGS) -c $< -o $@

# The entropy coder's serial chain uses lzcnt/tzcnt and shlx/shrx (x86-64-v3:
# the Xeon here and the GPU box's EPYC both have them): 9 % faster per frame.
$(OBJ)/entropy.o: $(SRC)/entropy.cpp $(HDRS)
	@mkdir -p $(OBJ)
	$(CXX) $(CXXFLAGS) -march=x86-64-v3 -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(dir $(LIB))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -lpthread

# A C++ caller of the drop-in evx1_encoder API (tests and bench.py's api_encode leg).
$(API_BIN): tests/api/evx1_api_caller.cpp include/evx1.h include/bitstream.h include/cairo_amd.h $(LIB)
	$(CXX) -O2 -std=c++17 -Wall -o $@ $< -L$(dir $(LIB)) -lcairo_amd -Wl,-rpath,'$$ORIGIN'

# Test infrastructure only (tests/, smoke(), bench.py cpu_baseline).  -O3 for
# x86-64-v3 (both hosts have it) halves the oracle's time per 4K frame, same bits.
$(ORACLE): oracle/evx_oracle.c oracle/evx_oracle.h
	gcc -O3 -march=x86-64-v3 -std=c11 -fPIC -shared -Wall -o $@ oracle/evx_oracle.c -lm

# Every build switch of the kernels that stays, compiled for gfx950 (no GPU
# needed): the time-accounting build, the traffic-attribution builds (tools
# builds only: without CAIRO_TOOLS_BUILD they must be refused), a larger
# launch cap.
KNOB_OBJ = build/knobs
check-knobs:
	@mkdir -p $(KNOB_OBJ)
	$(HIPCC) $(HIPFLAGS) -DCAIRO_ACCT=1 -c $(SRC)/kernels.hip -o $(KNOB_OBJ)/acct.o
	$(HIPCC) $(HIPFLAGS) -DCAIRO_TOOLS_BUILD -DCAIRO_ATTR_SKIP=1 -c $(SRC)/kernels.hip -o $(KNOB_OBJ)/attr1.o
	$(HIPCC) $(HIPFLAGS) -DCAIRO_TOOLS_BUILD -DCAIRO_ATTR_SKIP=4 -c $(SRC)/kernels.hip -o $(KNOB_OBJ)/attr4.o
	$(HIPCC) $(HIPFLAGS) -DCAIRO_TOOLS_BUILD -DCAIRO_ATTR_SKIP=120 -c $(SRC)/kernels.hip -o $(KNOB_OBJ)/attr120.o
	$(HIPCC) $(HIPFLAGS) -DCAIRO_MAX_BATCH=64 -c $(SRC)/kernels.hip -o $(KNOB_OBJ)/batch64.o
	$(HIPCC) $(HIPFLAGS) -DCAIRO_MAX_BATCH=64 -c $(SRC)/backend.hip -o $(KNOB_OBJ)/batch64_backend.o
	@if $(HIPCC) $(HIPFLAGS) -DCAIRO_ATTR_SKIP=1 -c $(SRC)/kernels.hip -o $(KNOB_OBJ)/refused.o 2>/dev/null; then \
	  echo "CAIRO_ATTR_SKIP without CAIRO_TOOLS_BUILD was not refused"; exit 1; fi
	@echo "check-knobs: every build switch compiles; CAIRO_ATTR_SKIP is refused in product builds"

clean:
	rm -rf build $(LIB) $(ORACLE) $(API_BIN) $(HOP_BIN)

.PHONY: all clean check-knobs
