# The reference's own applications, compiled UNMODIFIED from where they lie
# under /root/reference against this repository's ODP headers (include/) and
# linked to the product library (odp_amd/lib/libodpg.so): the drop-in check
# of SURVEY §8(f) rank 4. Outputs only into oracle/_ref/ (git-ignored; it
# travels to the GPU box like the built libraries). Nothing here is copied
# from the reference; without /root/reference this makefile does nothing.
# Usage: make -C oracle -f ref_apps.mk
REF     ?= /root/reference
CC      ?= gcc
OUT     := _ref
LIB     := $(abspath ../odp_amd/lib)
HDRS    := ../include/odp_api.h ../include/odp/rt.h ../include/odp/helper/odph_api.h \
	   ../include/odp_cls.h
LINK    := -L$(LIB) -lodpg -Wl,-rpath,'$$ORIGIN/../../odp_amd/lib' -L/opt/rocm/lib \
	   -Wl,-rpath,/opt/rocm/lib
APPS    := $(if $(wildcard $(REF)/example/classifier/odp_classifier.c),$(OUT)/odp_classifier) \
	   $(if $(wildcard $(REF)/test/performance/odp_bench_pktio_sp.c),$(OUT)/odp_bench_pktio_sp) \
	   $(if $(wildcard $(REF)/test/performance/odp_pktio_perf.c),$(OUT)/odp_pktio_perf)
# test/performance/odp_bench_pktio_sp.c with its two test/common sources
BENCH_SP := $(REF)/test/performance/odp_bench_pktio_sp.c $(REF)/test/common/bench_common.c \
	    $(REF)/test/common/export_results.c

all: $(APPS)

$(OUT)/odp_classifier: $(REF)/example/classifier/odp_classifier.c $(LIB)/libodpg.so $(HDRS)
	@mkdir -p $(OUT)
	$(CC) -std=gnu11 -O2 -Wall -I../include -o $@ $< $(LINK)

$(OUT)/odp_bench_pktio_sp: $(BENCH_SP) $(LIB)/libodpg.so $(HDRS)
	@mkdir -p $(OUT)
	$(CC) -std=gnu11 -O2 -Wall -I../include -I$(REF)/test/common -o $@ $(BENCH_SP) $(LINK)

# test/performance/odp_pktio_perf.c: the loop-pktio transmit -> receive
# throughput search
$(OUT)/odp_pktio_perf: $(REF)/test/performance/odp_pktio_perf.c $(LIB)/libodpg.so $(HDRS)
	@mkdir -p $(OUT)
	$(CC) -std=gnu11 -O2 -Wall -I../include -o $@ $< $(LINK)

clean:
	rm -rf $(OUT)/odp_classifier $(OUT)/odp_bench_pktio_sp $(OUT)/odp_pktio_perf

.PHONY: all clean
