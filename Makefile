# Sanitizer builds of the library's host code (ADVICE / VERDICT r1: ASan, UBSan,
# TSan over lt_lookup.cpp, lt_packer.cpp and the host half of lt_capi.cpp /
# lt_comm.cpp).  The host sources are compiled by g++ with the sanitizer; the
# device sources (lt_decode.hip, lt_results.hip) by hipcc for gfx950 without
# one (GPU sanitizers are not available on the pool).  The CPU test suite then
# runs against the instrumented library (LT_LIBRARY) with the sanitizer runtime
# preloaded into the interpreter:
#
#   make check-asan     # AddressSanitizer + UndefinedBehaviorSanitizer
#   make check-tsan     # ThreadSanitizer (threaded lattice builder and packer)
#
# The product library itself is built by `python -m lattice_based_tagger_amd._build`
# (or __graft_entry__.build()); `make lib` calls that.
ROCM ?= /opt/rocm
HIPCC ?= $(ROCM)/bin/hipcc
CXX := g++
PY ?= python3
CSRC := lattice_based_tagger_amd/csrc
OUT := build/san
HOST := lt_capi lt_packer lt_comm lt_lookup
DEV := lt_decode lt_results
HDRS := $(wildcard $(CSRC)/*.h) $(wildcard include/*.h)
SANFLAGS_COMMON := -O1 -g -std=c++17 -fPIC -ffp-contract=off -fno-omit-frame-pointer -Wall \
  -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include -Iinclude
ASAN := -fsanitize=address,undefined -fno-sanitize-recover=undefined
TSAN := -fsanitize=thread
LINK := -shared -L$(ROCM)/lib -lamdhip64 -ldl -Wl,-rpath,$(ROCM)/lib -Wl,--no-undefined
TESTS ?= tests
PYTEST := $(PY) -m pytest $(TESTS) -m "not gpu" -x -q -p no:cacheprovider
# TSan: a fork under the instrumented runtime can deadlock the child; the two
# suites that fork (nm of the library, gloo process groups) exercise no
# threaded host code of ours and run under ASan only
PYTEST_TSAN := $(PYTEST) --ignore=tests/test_capi.py --ignore=tests/test_dist.py

.PHONY: lib asan tsan check-asan check-tsan clean-san

lib:
	$(PY) -m lattice_based_tagger_amd._build

$(OUT)/dev/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -c $< -o $@

$(OUT)/asan/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(SANFLAGS_COMMON) $(ASAN) -c $< -o $@

$(OUT)/tsan/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(SANFLAGS_COMMON) $(TSAN) -c $< -o $@

$(OUT)/liblt_asan.so: $(HOST:%=$(OUT)/asan/%.o) $(DEV:%=$(OUT)/dev/%.o)
	$(CXX) $(ASAN) -o $@ $^ $(LINK)

$(OUT)/liblt_tsan.so: $(HOST:%=$(OUT)/tsan/%.o) $(DEV:%=$(OUT)/dev/%.o)
	$(CXX) $(TSAN) -o $@ $^ $(LINK)

asan: $(OUT)/liblt_asan.so
tsan: $(OUT)/liblt_tsan.so

# detect_leaks=0: the interpreter's own allocations are not ours to report
check-asan: asan
	LD_PRELOAD=$$($(CXX) -print-file-name=libasan.so) \
	ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
	UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
	LT_LIBRARY=$(abspath $(OUT)/liblt_asan.so) $(PYTEST)

check-tsan: tsan
	LD_PRELOAD=$$($(CXX) -print-file-name=libtsan.so) \
	TSAN_OPTIONS=halt_on_error=1:report_signal_unsafe=0 \
	LT_LIBRARY=$(abspath $(OUT)/liblt_tsan.so) $(PYTEST_TSAN)

clean-san:
	rm -rf $(OUT)
