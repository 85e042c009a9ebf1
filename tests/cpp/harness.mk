# tests/cpp/harness.mk -- builds the reference's own RS harnesses, unchanged, against the drop-in
# (include/ first on the include path, libezrs_hip.so / libezrs_fec.so as the engine).  Run by
# __graft_entry__.build() where /root/reference exists; the binaries land in tests/cpp/_bin/ and
# travel to the GPU box, where tests/test_ref_harness_gpu.py runs them.
#
#   rsexercise   rsexercise.C + exercise.H (ezpwd::RS<...>, the reed_solomon<7 params> type surface)
#   rsvalidate   rsvalidate.C: ezpwd::reed_solomon_base codecs on the engine, cross-checked against
#                Phil Karn's CPU libfec (oracle/_ref/libkarn.so, the reference's checker, built from
#                phil-karn/fec-3.0.1.tar.gz by oracle/Makefile)
#   rsspeed      rsspeed.C: the same pairing, timed (single-codeword calls)
#   rstest       phil-karn/rstest.c + exercise.c (x4: char, int, fixed-8, CCSDS), compiled with the
#                tarball's own headers, linked against libezrs_fec.so: Karn's ABI over the engine.
#                exercise.c is compiled with -DDEBUG=1, the reference's own knob that sets 10 trials
#                per (pad, load) class (exercise.c:136-138): rstest.c's Tab asks for up to 100000
#                single-codeword round trips per class, hours of PCIe round trips through a GPU
#
# The tarball is unpacked (headers only are used) into a temporary directory outside the repository,
# with the reference's int-symbol patch applied exactly as phil-karn/GNUmakefile:43-52 prepares it,
# and the directory is deleted when the recipe ends: no reference source stays under tests/ or
# travels to the GPU box.  Nothing from the reference is copied into the repository.
REFERENCE ?= /root/reference
HERE      := $(dir $(abspath $(lastword $(MAKEFILE_LIST))))
ROOT      := $(abspath $(HERE)../..)
OUT       := $(HERE)_bin
LIB       := $(ROOT)/ezpwd-reed-solomon_amd/lib
KARNLIB   := $(ROOT)/oracle/_ref
CXXF      := -std=c++17 -O2 -w -I$(ROOT)/include -I$(REFERENCE)/c++ -I$(REFERENCE)
TGZ       := $(REFERENCE)/phil-karn/fec-3.0.1.tar.gz
KEX       := $(REFERENCE)/phil-karn/exercise.c

.PHONY: all FORCE
all: $(OUT)/rsexercise $(OUT)/.karn_stamp
FORCE:

# the stamp stands for three binaries: if any of them is gone (a partial clean of _bin), rebuild
KARN_BINS    := $(OUT)/rsvalidate $(OUT)/rsspeed $(OUT)/rstest
KARN_MISSING := $(filter-out $(wildcard $(KARN_BINS)),$(KARN_BINS))

$(OUT)/rsexercise: $(REFERENCE)/rsexercise.C $(REFERENCE)/exercise.H $(ROOT)/include/ezpwd_amd/rs
	@mkdir -p $(OUT)
	g++ $(CXXF) -o $@ $< -L$(LIB) -lezrs_hip -Wl,-rpath,$(LIB)

# rsvalidate, rsspeed and rstest: the programs that need libfec's headers, built in one recipe around
# one temporary unpack of the tarball
$(OUT)/.karn_stamp: $(REFERENCE)/rsvalidate.C $(REFERENCE)/rsspeed.C $(REFERENCE)/phil-karn/rstest.c $(KEX) \
                    $(TGZ) $(ROOT)/include/ezpwd_amd/rs $(LIB)/libezrs_fec.so $(HERE)harness.mk \
                    $(if $(KARN_MISSING),FORCE)
	@mkdir -p $(OUT)
	@rm -rf $(OUT)/.fec $(OUT)/.o
	T=$$(mktemp -d /tmp/ezrs_fec.XXXXXX) && ( set -e; \
	  tar xzf $(TGZ) -C $$T; \
	  cd $$T/fec-3.0.1 && for p in $(REFERENCE)/phil-karn/fec-3.0.1*.patch; do patch -s -p1 < $$p; done; \
	  ln -sfn fec-3.0.1 $$T/fec; \
	  KF="-I$(REFERENCE)/phil-karn -I$$T"; \
	  g++ $(CXXF) $$KF -o $(OUT)/rsvalidate $(REFERENCE)/rsvalidate.C -L$(LIB) -lezrs_hip -L$(KARNLIB) -lkarn \
	      -Wl,-rpath,$(LIB) -Wl,-rpath,$(KARNLIB); \
	  g++ $(CXXF) $$KF -o $(OUT)/rsspeed $(REFERENCE)/rsspeed.C -L$(LIB) -lezrs_hip -L$(KARNLIB) -lkarn \
	      -Wl,-rpath,$(LIB) -Wl,-rpath,$(KARNLIB); \
	  KC="-O2 -w -I$$T/fec-3.0.1 $$KF"; \
	  gcc $$KC -c -o $$T/rstest.o $(REFERENCE)/phil-karn/rstest.c; \
	  gcc $$KC -DDEBUG=1 -c -o $$T/ex_char.o $(KEX); \
	  gcc $$KC -DDEBUG=1 -DBIGSYM -c -o $$T/ex_int.o $(KEX); \
	  gcc $$KC -DDEBUG=1 -DFIXED -c -o $$T/ex_8.o $(KEX); \
	  gcc $$KC -DDEBUG=1 -DCCSDS -c -o $$T/ex_ccsds.o $(KEX); \
	  g++ -o $(OUT)/rstest $$T/rstest.o $$T/ex_char.o $$T/ex_int.o $$T/ex_8.o $$T/ex_ccsds.o \
	      -L$(LIB) -lezrs_fec -lezrs_hip -Wl,-rpath,$(LIB) ); rc=$$?; rm -rf $$T; exit $$rc
	touch $@
