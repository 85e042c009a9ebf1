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
# The tarball is unpacked (headers only are used) into a scratch directory with the reference's
# int-symbol patch applied, exactly as phil-karn/GNUmakefile:43-52 prepares it.  Nothing from the
# reference is copied into the repository.
REFERENCE ?= /root/reference
HERE      := $(dir $(abspath $(lastword $(MAKEFILE_LIST))))
ROOT      := $(abspath $(HERE)../..)
OUT       := $(HERE)_bin
LIB       := $(ROOT)/ezpwd-reed-solomon_amd/lib
KARNLIB   := $(ROOT)/oracle/_ref
FECDIR    := $(OUT)/.fec
CXXF      := -std=c++17 -O2 -w -I$(ROOT)/include -I$(REFERENCE)/c++ -I$(REFERENCE)
KARNF     := -I$(REFERENCE)/phil-karn -I$(FECDIR)

.PHONY: all
all: $(OUT)/rsexercise $(OUT)/rsvalidate $(OUT)/rsspeed $(OUT)/rstest

$(FECDIR)/fec/fec.h: $(REFERENCE)/phil-karn/fec-3.0.1.tar.gz
	rm -rf $(FECDIR) && mkdir -p $(FECDIR)
	tar xzf $< -C $(FECDIR)
	cd $(FECDIR)/fec-3.0.1 && for p in $(REFERENCE)/phil-karn/fec-3.0.1*.patch; do patch -s -p1 < $$p; done
	ln -sfn fec-3.0.1 $(FECDIR)/fec
	touch $@

$(OUT)/rsexercise: $(REFERENCE)/rsexercise.C $(REFERENCE)/exercise.H $(ROOT)/include/ezpwd_amd/rs
	@mkdir -p $(OUT)
	g++ $(CXXF) -o $@ $< -L$(LIB) -lezrs_hip -Wl,-rpath,$(LIB)

$(OUT)/rsvalidate: $(REFERENCE)/rsvalidate.C $(ROOT)/include/ezpwd_amd/rs $(FECDIR)/fec/fec.h
	@mkdir -p $(OUT)
	g++ $(CXXF) $(KARNF) -o $@ $< -L$(LIB) -lezrs_hip -L$(KARNLIB) -lkarn -Wl,-rpath,$(LIB) -Wl,-rpath,$(KARNLIB)

$(OUT)/rsspeed: $(REFERENCE)/rsspeed.C $(ROOT)/include/ezpwd_amd/rs $(FECDIR)/fec/fec.h
	@mkdir -p $(OUT)
	g++ $(CXXF) $(KARNF) -o $@ $< -L$(LIB) -lezrs_hip -L$(KARNLIB) -lkarn -Wl,-rpath,$(LIB) -Wl,-rpath,$(KARNLIB)

KEX := $(REFERENCE)/phil-karn/exercise.c
KCF := -O2 -w -I$(FECDIR)/fec-3.0.1 $(KARNF)
KXF := $(KCF) -DDEBUG=1
$(OUT)/rstest: $(REFERENCE)/phil-karn/rstest.c $(KEX) $(FECDIR)/fec/fec.h $(LIB)/libezrs_fec.so
	@mkdir -p $(OUT)/.o
	gcc $(KCF) -c -o $(OUT)/.o/rstest.o $(REFERENCE)/phil-karn/rstest.c
	gcc $(KXF) -c -o $(OUT)/.o/exercise_char.o $(KEX)
	gcc $(KXF) -DBIGSYM -c -o $(OUT)/.o/exercise_int.o $(KEX)
	gcc $(KXF) -DFIXED -c -o $(OUT)/.o/exercise_8.o $(KEX)
	gcc $(KXF) -DCCSDS -c -o $(OUT)/.o/exercise_ccsds.o $(KEX)
	g++ -o $@ $(OUT)/.o/rstest.o $(OUT)/.o/exercise_char.o $(OUT)/.o/exercise_int.o \
	    $(OUT)/.o/exercise_8.o $(OUT)/.o/exercise_ccsds.o -L$(LIB) -lezrs_fec -lezrs_hip -Wl,-rpath,$(LIB)
