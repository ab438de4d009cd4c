# ref.mk — recipe that compiles the reference's own nanopb runtime and its
# generated ip.pb.c IN PLACE from /root/reference (nothing is copied) into
# oracle/_ref/libnanopb_ref.so, together with the application callback the
# firmware would supply (nanopb_ref_harness.c).  TEST INFRASTRUCTURE ONLY.
#
#   make -f oracle/ref.mk            (from the repo root)
#
# libopus (hardware/lib/libopus/src) is NOT built: celt/cwrs.c:38,
# silk/VAD.c:31 and silk/sigm_Q15.c:31 include the ESP32 <pgmspace.h>, which
# this image lacks; building it would need a stand-in header, so it is treated
# as unbuildable here.

REF      ?= /root/reference
NANOPB   := $(REF)/hardware/lib/nanopb/src
PROTOGEN := $(REF)/hardware/src/protogen
OUT      := oracle/_ref
SRCS     := $(NANOPB)/pb_common.c $(NANOPB)/pb_encode.c $(NANOPB)/pb_decode.c \
            $(PROTOGEN)/ip.pb.c oracle/nanopb_ref_harness.c

all: $(OUT)/libnanopb_ref.so

$(OUT)/libnanopb_ref.so: $(SRCS)
	@mkdir -p $(OUT)
	gcc -O2 -fPIC -shared -I$(NANOPB) -I$(PROTOGEN) $(SRCS) -o $@

clean:
	rm -f $(OUT)/libnanopb_ref.so

.PHONY: all clean
