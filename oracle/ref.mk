# oracle/ref.mk -- TEST INFRASTRUCTURE ONLY.
#
# Compiles the reference GMAP 2024-02-22 C sources *where they lie* under
# $(REF)/src into oracle/_ref/ (git-ignored; it travels to the GPU box with the
# gpurun snapshot like any other built .so).  Nothing under /root/reference is
# copied into the repository and the reference's own build system (autotools)
# is not run: the source list is GMAP_FILES from src/Makefile.am:226-265 and
# the per-variant SIMD defines are those of src/Makefile.am:268-319.  The
# reference ships its own src/config.h, which is used as-is.
#
# That shipped config.h was generated on the upstream author's macOS machine:
# it sets HAVE_BZLIB (no <bzlib.h> here) and PAGESIZE_VIA_SYSCTL (macOS-only
# <sys/sysctl.h>).  bzip2.c and getline.c use config.h only for HAVE_BZLIB, so
# they are compiled without -DHAVE_CONFIG_H (their own no-bzip2 configuration).
# access.c uses config.h for PAGESIZE_VIA_SYSCTL (<sys/sysctl.h>, macOS-only)
# and mmap/shm feature switches, so it is compiled WITHOUT config.h, with the
# Linux values of the switches it reads given as -D flags (ACCESS_DEFS below;
# the same values `./configure` reports on this image, config.log).  The
# harness library does not need access.c (it links with --gc-sections and
# exports only refh_*); the full `gmap` programs below do.
#
# Products (per variant V in {nosimd, avx2}):
#   _ref/V/*.o                 reference objects
#   _ref/librefdp_V.so         reference objects + refharness.c: a flat C API
#                              over the reference's own Dynprog_* entry points,
#                              used only by tests/ and the golden generator.
#   _ref/gmap_V                the reference `gmap` program itself (all of
#                              GMAP_FILES, unmodified): the end-to-end oracle
#   _ref/gmap_large            gmapl (the nosimd build with LARGE_GENOMES: 64-bit Univcoord_T), and
#   _ref/gmap_gpu_large        gmapl linked with the drop-in shim
#   _ref/gmap_gpu_V            the same objects linked with the drop-in shim
#                              (`ld --wrap`) and libgmapdp.so:
#                              GMAP's own per-read pipeline on the MI355X engine

REF      ?= /root/reference
SRC      := $(REF)/src
OUT      ?= _ref
CC       := gcc
BASEFLAGS := -O3 -fomit-frame-pointer -fPIC -pthread -I$(SRC) \
             -DTARGET=\"x86_64-pc-linux-gnu\" -DGMAPDB=\"/nonexistent/gmapdb\" -w \
             -ffunction-sections -fdata-sections

GMAP_C := except.c assert.c mem.c intlist.c uintlist.c list.c littleendian.c bigendian.c \
  univinterval.c interval.c stopwatch.c semaphore.c access.c filestring.c iit-read-univ.c \
  iit-read.c md5.c bzip2.c fopen.c sequence.c reader.c genomicpos.c compress.c compress-write.c \
  gbuffer.c genome.c popcount.c dinucl_bits.c genome_canonical.c genome-write.c bitpack64-read.c \
  bitpack64-readtwo.c indexdb.c oligo.c block.c chrom.c segmentpos.c chrnum.c uinttable_rh.c \
  gregion.c match.c matchpool.c diagnostic.c stage1.c diag.c diagpool.c cmet.c atoi.c orderstat.c \
  oligoindex_hr.c intron.c maxent.c maxent_hr.c pair.c pairpool.c cellpool.c stage2.c doublelist.c \
  smooth.c splicestringpool.c splicetrie_build.c splicetrie.c boyer-moore.c dynprog.c dynprog_simd.c \
  dynprog_single.c dynprog_genome.c dynprog_cdna.c dynprog_end.c translation.c pbinom.c \
  changepoint.c stage3.c request.c result.c output.c inbuffer.c samheader.c printbuffer.c \
  outbuffer.c chimera.c datadir.c parserange.c getline.c getopt.c getopt1.c gmap.c

# Not buildable with the shipped (macOS) config.h: compiled with ACCESS_DEFS instead.
UNBUILDABLE_C := access.c
ACCESS_DEFS := -DHAVE_UNISTD_H=1 -DHAVE_SYS_TYPES_H=1 -DHAVE_STDDEF_H=1 -DHAVE_SYS_STAT_H=1 -DHAVE_FCNTL_H=1 \
  -DHAVE_STDINT_H=1 -DHAVE_INTTYPES_H=1 -DHAVE_INLINE=1 -DHAVE_PTHREAD=1 -DPAGESIZE_VIA_SYSCONF=1 -DHAVE_SYSCONF=1 \
  -DHAVE_MMAP=1 -DHAVE_MUNMAP=1 -DHAVE_MMAP_MAP_PRIVATE=1 -DHAVE_MMAP_MAP_FILE=1 -DHAVE_MMAP_MAP_SHARED=1 \
  -DHAVE_CADDR_T=1 -DHAVE_MADVISE=1 -DHAVE_MADVISE_MADV_RANDOM=1 -DHAVE_MADVISE_MADV_DONTNEED=1 \
  -DHAVE_MADVISE_MADV_WILLNEED=1 -DHAVE_MADVISE_MADV_SEQUENTIAL=1 -DHAVE_SHMAT=1 -DHAVE_SHMGET=1 -DHAVE_SHMCTL=1 \
  -DHAVE_SHMDT=1 -DHAVE_SEMCTL=1 -DHAVE_SEMGET=1 -DHAVE_SEMOP=1 -DHAVE_STAT64=1 \
  -DSIZEOF_UNSIGNED_LONG=8 -DSIZEOF_UNSIGNED_LONG_LONG=8 -DSIZEOF_OFF_T=8
# Compiled without config.h (their only config switch is HAVE_BZLIB).
NOCONFIG_C := bzip2.c getline.c
# Driver (main) and output/threading layers: not linked into the harness.
NOTLINKED_C := gmap.c inbuffer.c outbuffer.c
HARNESS_C := $(filter-out $(UNBUILDABLE_C) $(NOTLINKED_C),$(GMAP_C))

FLAGS_nosimd :=
FLAGS_avx2   := -mpopcnt -DHAVE_SSE2=1 -DHAVE_SSSE3=1 -DHAVE_SSE4_1=1 -DHAVE_SSE4_2=1 -DHAVE_AVX2=1 \
                -msse2 -mssse3 -msse4.1 -msse4.2 -mavx2 -mno-avx512f -mno-avx512cd -mno-avx512vl -mno-avx512bw

# nosimd built as `./configure --enable-alloca` would (configure.ac:220-228,
# AC_FUNC_ALLOCA on glibc): MALLOCA/FREEA become alloca/no-op (mem.h:97-116).
# Only used to pin Dynprog_genome_gap with halfp, where the default heap build
# dereferences the FREEA-nulled leftdi (dynprog_genome.c:2879-2888) and crashes.
FLAGS_nosimda := -DHAVE_ALLOCA=1 -DHAVE_ALLOCA_H=1
# The same for the AVX2 build (bridge_intron_gap_8/16_site_level reads leftdi after FREEA too,
# dynprog_genome.c:1370-1379 / :2245-2254).
FLAGS_avx2a  := $(FLAGS_avx2) -DHAVE_ALLOCA=1 -DHAVE_ALLOCA_H=1
# gmapl: the nosimd build with 64-bit Univcoord_T (src/Makefile.am:366, -DLARGE_GENOMES=1) and the two
# extra sources of GMAPL_FILES (src/Makefile.am:324).
FLAGS_large  := -DLARGE_GENOMES=1
SRCS_large   := $(GMAP_C) uint8list.c uint8table_rh.c

.DEFAULT_GOAL := all

VARIANTS := nosimd avx2 nosimda avx2a large

define variant_rules
LIBOBJS_$(1) := $$(patsubst %.c,$(OUT)/$(1)/%.o,$$(filter-out $(UNBUILDABLE_C) $(NOTLINKED_C),$$(or $$(SRCS_$(1)),$(GMAP_C))))

$(OUT)/$(1)/%.o: $(SRC)/%.c
	@mkdir -p $$(dir $$@)
	$$(CC) $(BASEFLAGS) $$(if $$(filter $$(notdir $$<),$(NOCONFIG_C)),,-DHAVE_CONFIG_H) $$(FLAGS_$(1)) -c $$< -o $$@

$(OUT)/$(1)/refharness.o: refharness.c
	@mkdir -p $$(dir $$@)
	$$(CC) $(BASEFLAGS) -DHAVE_CONFIG_H $$(FLAGS_$(1)) -I. -c $$< -o $$@

$(OUT)/librefdp_$(1).so: $$(LIBOBJS_$(1)) $(OUT)/$(1)/refharness.o
	$$(CC) -shared -pthread -Wl,--gc-sections -Wl,--version-script=refharness.map -o $$@ $$^ -lz -lm

$(OUT)/$(1)/access.o: $(SRC)/access.c
	@mkdir -p $$(dir $$@)
	$$(CC) $(BASEFLAGS) $(ACCESS_DEFS) $$(FLAGS_$(1)) -c $$< -o $$@

PROGOBJS_$(1) := $$(patsubst %.c,$(OUT)/$(1)/%.o,$$(or $$(SRCS_$(1)),$(GMAP_C)))
endef

$(foreach v,$(VARIANTS),$(eval $(call variant_rules,$(v))))

# iit_store (src/Makefile.am IIT_STORE_FILES), the reference's own IIT writer: it builds the known
# splice-site file of the `gmap -s` end-to-end test (tests/golden/make_e2e.py) from a text list.
IIT_STORE_C := except.c assert.c mem.c intlist.c list.c littleendian.c bigendian.c univinterval.c interval.c \
  uintlist.c stopwatch.c semaphore.c access.c doublelist.c iit-write-univ.c iit-write.c tableint.c table.c \
  chrom.c bzip2.c getline.c getopt.c getopt1.c iit_store.c
$(OUT)/iit_store: $(patsubst %.c,$(OUT)/nosimd/%.o,$(IIT_STORE_C))
	$(CC) -pthread -o $@ $^ -lz -lm

# gmapindex (src/Makefile.am GMAPINDEX_FILES, built with -DUTILITYP=1 as gmapindex_CFLAGS says) and
# the reference's gmap_build / fa_coords / gmap_process perl scripts (util/) make the small indexed
# genome of the `gmap -d` / `gmap -d -s` end-to-end fixtures (tests/golden/make_index.py).
FLAGS_util := -DUTILITYP=1
$(eval $(call variant_rules,util))
GMAPINDEX_C := except.c assert.c mem.c intlist.c list.c littleendian.c bigendian.c univinterval.c interval.c \
  uintlist.c stopwatch.c semaphore.c access.c filestring.c iit-read-univ.c iit-write-univ.c iit-read.c md5.c \
  bzip2.c fopen.c sequence.c genome.c genomicpos.c compress-write.c genome-write.c compress.c popcount.c \
  bitpack64-read.c bitpack64-readtwo.c bitpack64-access.c bitpack64-incr.c bitpack64-write.c indexdb.c \
  indexdb-write.c saca-k.c localdb-write.c table.c tableuint.c tableuint8.c tableint.c bytecoding.c \
  sarray-write.c chrom.c segmentpos.c uint8list.c parserange.c getline.c gmapindex.c
$(OUT)/bin/gmapindex: $(patsubst %.c,$(OUT)/util/%.o,$(GMAPINDEX_C))
	@mkdir -p $(dir $@)
	$(CC) -pthread -o $@ $^ -lz -lm
$(OUT)/bin/iit_store: $(OUT)/iit_store
	@mkdir -p $(dir $@)
	cp $< $@
index_tools: $(OUT)/bin/gmapindex $(OUT)/bin/iit_store

SHIM_SRC   := ../gmap-2024_amd/shim/gmapdp_gmap_shim.c
GMAPDP_LIB := ../gmap-2024_amd/lib

all: programs $(OUT)/iit_store $(foreach v,$(VARIANTS),$(OUT)/librefdp_$(v).so) \
     $(if $(wildcard $(GMAPDP_LIB)/libgmapdp.so),$(OUT)/librefdp_gpushim.so $(OUT)/librefdp_gpushim_avx2.so)

# The drop-in check: the same nosimd reference objects, with Dynprog_init / _*_setup /
# _single_gap / _end5_gap / _end3_gap / _genome_gap routed by `ld --wrap` to the engine's
# GMAP shim (gmap-2024_amd/shim, compiled against the reference's headers exactly as a GMAP
# build would) and libgmapdp.so.  Tests call it through the same refh_* entry points.
WRAPPED    := Dynprog_init Dynprog_single_setup Dynprog_end_setup Dynprog_genome_setup \
              Dynprog_single_gap Dynprog_end5_gap Dynprog_end3_gap Dynprog_genome_gap Dynprog_cdna_gap \
              Dynprog_microexon_int Oligoindex_hr_tally Oligoindex_get_mappings Stage2_setup Stage2_compute \
              Dynprog_end5_splicejunction Dynprog_end3_splicejunction Dynprog_end5_known Dynprog_end3_known

$(OUT)/gpushim/gmapdp_gmap_shim.o: $(SHIM_SRC) ../include/gmapdp.h
	@mkdir -p $(dir $@)
	$(CC) $(BASEFLAGS) -DHAVE_CONFIG_H -I../include -c $< -o $@

$(OUT)/librefdp_gpushim.so: $(LIBOBJS_nosimd) $(OUT)/nosimd/refharness.o $(OUT)/gpushim/gmapdp_gmap_shim.o \
                            $(GMAPDP_LIB)/libgmapdp.so
	$(CC) -shared -pthread -Wl,--gc-sections -Wl,--version-script=refharness.map \
	  $(foreach w,$(WRAPPED),-Wl,--wrap=$(w)) -o $@ $(filter %.o,$^) \
	  -L$(GMAPDP_LIB) -lgmapdp -Wl,-rpath,'$$ORIGIN/../../gmap-2024_amd/lib' -lz -lm

# The same drop-in inside a SIMD build: the AVX2 objects (alloca variant, see FLAGS_avx2a) and the
# shim compiled with the AVX2 build's defines, so every call carries GMAPDP_SIMD.
$(OUT)/gpushim_avx2/gmapdp_gmap_shim.o: $(SHIM_SRC) ../include/gmapdp.h
	@mkdir -p $(dir $@)
	$(CC) $(BASEFLAGS) -DHAVE_CONFIG_H $(FLAGS_avx2a) -I../include -c $< -o $@

$(OUT)/librefdp_gpushim_avx2.so: $(LIBOBJS_avx2a) $(OUT)/avx2a/refharness.o $(OUT)/gpushim_avx2/gmapdp_gmap_shim.o \
                                 $(GMAPDP_LIB)/libgmapdp.so
	$(CC) -shared -pthread -Wl,--gc-sections -Wl,--version-script=refharness.map \
	  $(foreach w,$(WRAPPED),-Wl,--wrap=$(w)) -o $@ $(filter %.o,$^) \
	  -L$(GMAPDP_LIB) -lgmapdp -Wl,-rpath,'$$ORIGIN/../../gmap-2024_amd/lib' -lz -lm

# ---- the full gmap program (end-to-end oracle) and the same program on the MI355X engine ----
# gmap_gpu_V owns the whole Dynprog_* interface (SURVEY §8b's unit of replacement): the six dynprog*.o
# objects are NOT linked; the shim, compiled with -DGMAPDP_SHIM_OWN, defines all 21 Dynprog_* symbols GMAP
# imports.  Only the stage-2 pair is still routed with --wrap (stage2.o / oligoindex_hr.o stay linked for
# their other entry points).
DYNPROG_C   := dynprog.c dynprog_simd.c dynprog_single.c dynprog_genome.c dynprog_cdna.c dynprog_end.c
WRAPPED_OWN := Oligoindex_hr_tally Oligoindex_get_mappings Stage2_setup Stage2_compute \
               pthread_create pthread_join pthread_getspecific pthread_setspecific
PROG_VARIANTS := nosimd avx2 large
define prog_rules
$(OUT)/gmap_$(1): $$(PROGOBJS_$(1))
	$$(CC) -pthread -s -o $$@ $$^ -lz -lm

NODP_$(1) := $$(filter-out $$(patsubst %.c,$(OUT)/$(1)/%.o,$(DYNPROG_C)),$$(PROGOBJS_$(1)))

$(OUT)/gmap_gpu_$(1): $$(NODP_$(1)) $(OUT)/gpushim_own_$(1)/gmapdp_gmap_shim.o $(GMAPDP_LIB)/libgmapdp.so
	$$(CC) -pthread -s $(foreach w,$(WRAPPED_OWN),-Wl,--wrap=$(w)) -o $$@ $$(filter %.o,$$^) \
	  -L$(GMAPDP_LIB) -lgmapdp -Wl,-rpath,'$$$$ORIGIN/../../gmap-2024_amd/lib' -lz -lm

$(OUT)/gpushim_own_$(1)/gmapdp_gmap_shim.o: $(SHIM_SRC) ../include/gmapdp.h ../include/gmapdp_dynprog.h
	@mkdir -p $$(dir $$@)
	$$(CC) $(BASEFLAGS) -DHAVE_CONFIG_H -DGMAPDP_SHIM_OWN $$(FLAGS_$(1)) -I../include -c $$< -o $$@

# the same two programs unstripped, with the sampling profiler (tools/pcprof.c, idle unless PCPROF_OUT is set)
$(OUT)/gmap_prof_$(1): $$(PROGOBJS_$(1)) $(OUT)/pcprof.o
	$$(CC) -pthread -o $$@ $$^ -lz -lm

$(OUT)/gmap_gpu_prof_$(1): $$(NODP_$(1)) $(OUT)/gpushim_own_$(1)/gmapdp_gmap_shim.o $(OUT)/pcprof.o $(GMAPDP_LIB)/libgmapdp.so
	$$(CC) -pthread $(foreach w,$(WRAPPED_OWN),-Wl,--wrap=$(w)) -o $$@ $$(filter %.o,$$^) \
	  -L$(GMAPDP_LIB) -lgmapdp -Wl,-rpath,'$$$$ORIGIN/../../gmap-2024_amd/lib' -lz -lm
endef

$(OUT)/pcprof.o: ../tools/pcprof.c
	@mkdir -p $(dir $@)
	$(CC) -O2 -g -c $< -o $@
$(foreach v,$(PROG_VARIANTS),$(eval $(call prog_rules,$(v))))

# own_check (tests/test_shim_own.py): the non-DP Dynprog_* entry points (consistent table, scores, handles)
# from the reference's dynprog objects and from the owned shim, printed for comparison; no GPU call.
$(OUT)/nosimd/own_check.o: own_check.c
	@mkdir -p $(dir $@)
	$(CC) $(BASEFLAGS) -DHAVE_CONFIG_H -c $< -o $@
$(OUT)/own_check_ref: $(filter-out $(OUT)/nosimd/gmap.o,$(PROGOBJS_nosimd)) $(OUT)/nosimd/own_check.o
	$(CC) -pthread -o $@ $^ -lz -lm
$(OUT)/own_check_shim: $(filter-out $(OUT)/nosimd/gmap.o,$(NODP_nosimd)) $(OUT)/gpushim_own_nosimd/gmapdp_gmap_shim.o \
                       $(OUT)/nosimd/own_check.o $(GMAPDP_LIB)/libgmapdp.so
	$(CC) -pthread $(foreach w,$(WRAPPED_OWN),-Wl,--wrap=$(w)) -o $@ $(filter %.o,$^) \
	  -L$(GMAPDP_LIB) -lgmapdp -Wl,-rpath,'$$ORIGIN/../../gmap-2024_amd/lib' -lz -lm
# fiber_check: the drop-in's worker fibers (pthread_* wrapped as in gmap_gpu_*) without a GPU
$(OUT)/nosimd/fiber_check.o: fiber_check.c
	@mkdir -p $(dir $@)
	$(CC) $(BASEFLAGS) -c $< -o $@
$(OUT)/fiber_check: $(filter-out $(OUT)/nosimd/gmap.o,$(NODP_nosimd)) $(OUT)/gpushim_own_nosimd/gmapdp_gmap_shim.o \
                    $(OUT)/nosimd/fiber_check.o $(GMAPDP_LIB)/libgmapdp.so
	$(CC) -pthread $(foreach w,$(WRAPPED_OWN),-Wl,--wrap=$(w)) -o $@ $(filter %.o,$^) \
	  -L$(GMAPDP_LIB) -lgmapdp -Wl,-rpath,'$$ORIGIN/../../gmap-2024_amd/lib' -lz -lm
own_check: $(OUT)/own_check_ref $(if $(wildcard $(GMAPDP_LIB)/libgmapdp.so),$(OUT)/own_check_shim $(OUT)/fiber_check)

programs: $(foreach v,$(PROG_VARIANTS),$(OUT)/gmap_$(v)) $(OUT)/gmap_callmix own_check $(OUT)/gmap_prof_nosimd \
          $(if $(wildcard $(GMAPDP_LIB)/libgmapdp.so),$(foreach v,$(PROG_VARIANTS),$(OUT)/gmap_gpu_$(v)) $(OUT)/gmap_gpu_prof_nosimd)

# The unmodified nosimd gmap with the hot-path entry points counted (callmix.c: one log line per call,
# then the reference's own function): the measured per-read call mix of a read shape (tools/callmix.py)
CALLMIX := Dynprog_single_gap Dynprog_end5_gap Dynprog_end3_gap Dynprog_genome_gap Dynprog_cdna_gap \
           Dynprog_microexon_int Stage2_compute Oligoindex_get_mappings
$(OUT)/callmix/callmix.o: callmix.c ../include/gmapdp_dynprog.h
	@mkdir -p $(dir $@)
	$(CC) $(BASEFLAGS) -DHAVE_CONFIG_H -I../include -c $< -o $@

$(OUT)/gmap_callmix: $(PROGOBJS_nosimd) $(OUT)/callmix/callmix.o
	$(CC) -pthread -s $(foreach w,$(CALLMIX),-Wl,--wrap=$(w)) -o $@ $^ -lz -lm

.PHONY: all programs own_check
