# ref.mk — recipe that compiles the reference's own nanopb runtime and its
# generated ip.pb.c IN PLACE from /root/reference (nothing is copied) into
# oracle/_ref/libnanopb_ref.so, together with the application callback the
# firmware would supply (nanopb_ref_harness.c).  TEST INFRASTRUCTURE ONLY.
#
#   make -f oracle/ref.mk            (from the repo root)
#
# It also compiles the reference's own FFT (libopus celt/kiss_fft.c, the
# static mode tables of celt/modes.c and celt/mathops.c, with the reference's
# own config.h: FIXED_POINT, no CUSTOM_MODES) into oracle/_ref/
# libkissfft_ref.so together with kissfft_ref_harness.c. These three files
# compile from the reference's own headers. The rest of libopus is NOT built:
# celt/cwrs.c:38, silk/VAD.c:31 and silk/sigm_Q15.c:31 include the ESP32
# <pgmspace.h>, which this image lacks; building them would need a stand-in
# header, so the full library is treated as unbuildable here.

REF      ?= /root/reference
NANOPB   := $(REF)/hardware/lib/nanopb/src
PROTOGEN := $(REF)/hardware/src/protogen
OUT      := oracle/_ref
SRCS     := $(NANOPB)/pb_common.c $(NANOPB)/pb_encode.c $(NANOPB)/pb_decode.c \
            $(PROTOGEN)/ip.pb.c oracle/nanopb_ref_harness.c

OPUS     := $(REF)/hardware/lib/libopus/src
KF_SRCS  := $(OPUS)/celt/kiss_fft.c $(OPUS)/celt/modes.c $(OPUS)/celt/mathops.c \
            oracle/kissfft_ref_harness.c

KC_SRCS  := $(OPUS)/celt/kiss_fft.c $(OPUS)/celt/mathops.c oracle/kissfft_custom_harness.c

all: $(OUT)/libnanopb_ref.so $(OUT)/libkissfft_ref.so $(OUT)/libkissfft_custom.so

$(OUT)/libkissfft_ref.so: $(KF_SRCS)
	@mkdir -p $(OUT)
	gcc -O2 -fPIC -shared -DHAVE_CONFIG_H -I$(OPUS) -I$(OPUS)/celt $(KF_SRCS) -o $@ \
	    -Wl,--no-undefined -lm

# the same kiss_fft.c with the libopus configure option CUSTOM_MODES on, so it
# allocates nfft = 1024 (kissfft_custom_harness.c); config.h otherwise unchanged
$(OUT)/libkissfft_custom.so: $(KC_SRCS)
	@mkdir -p $(OUT)
	gcc -O2 -fPIC -shared -DHAVE_CONFIG_H -DCUSTOM_MODES -I$(OPUS) -I$(OPUS)/celt $(KC_SRCS) -o $@ \
	    -Wl,--no-undefined -lm

$(OUT)/libnanopb_ref.so: $(SRCS)
	@mkdir -p $(OUT)
	gcc -O2 -fPIC -shared -I$(NANOPB) -I$(PROTOGEN) $(SRCS) -o $@

clean:
	rm -f $(OUT)/libnanopb_ref.so $(OUT)/libkissfft_ref.so $(OUT)/libkissfft_custom.so

.PHONY: all clean
