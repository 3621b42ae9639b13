# Builds the REFERENCE verifiers from their own sources under /root/reference into oracle/_ref/.
# These are test infrastructure only (golden-vector generation and the cpu_baseline leg of bench.py);
# nothing in dprf_amd/ links or loads them.  Sources are compiled where they lie; nothing is copied.
#
#   make -f oracle/ref.mk            (from the repo root)
#
# System OpenSSL (libcrypto 3.x, present in this image) provides the primitives the reference calls.
# RC4 lives in OpenSSL 3's legacy provider: run the executables with OPENSSL_CONF=oracle/openssl_legacy.cnf,
# or call ref_load_legacy() (ref_providers.c) before using the in-process libraries.
REF    ?= /root/reference/src
OUT    ?= oracle/_ref
CC     ?= gcc
CFLAGS ?= -O2 -w
LIBS   := -lssl -lcrypto

OFFICE := $(REF)/ms-offcrypto-impl/msoffcrypto_password_verifier.c
ODT    := $(REF)/odt-impl/odt_password_verifier.c
PDF    := $(REF)/pdf-impl/pdf_password_verifier.c

all: $(OUT)/msoffcrypto $(OUT)/odt $(OUT)/pdf \
     $(OUT)/libref_office.so $(OUT)/libref_odt.so $(OUT)/libref_pdf.so

$(OUT):
	mkdir -p $(OUT)

# argv-compatible executables: exactly what brute_force.py Popen()s (brute_force.py:163-197)
$(OUT)/msoffcrypto: $(OFFICE) | $(OUT)
	$(CC) $(CFLAGS) -o $@ $< $(LIBS)
$(OUT)/odt: $(ODT) | $(OUT)
	$(CC) $(CFLAGS) -o $@ $< $(LIBS)
$(OUT)/pdf: $(PDF) | $(OUT)
	$(CC) $(CFLAGS) -o $@ $< $(LIBS)

# in-process variants: the reference verify() with main renamed, for the CPU baseline (no fork/exec)
$(OUT)/libref_office.so: $(OFFICE) | $(OUT)
	$(CC) $(CFLAGS) -fPIC -shared -Dmain=ref_main -o $@ $< $(LIBS)
$(OUT)/libref_odt.so: $(ODT) | $(OUT)
	$(CC) $(CFLAGS) -fPIC -shared -Dmain=ref_main -o $@ $< $(LIBS)
$(OUT)/libref_pdf.so: $(PDF) oracle/ref_providers.c | $(OUT)
	$(CC) $(CFLAGS) -fPIC -shared -Dmain=ref_main -o $@ $(PDF) oracle/ref_providers.c $(LIBS)

clean:
	rm -rf $(OUT)
.PHONY: all clean
