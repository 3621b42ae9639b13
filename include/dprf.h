/* dprf.h -- C ABI of libdprf.so, the MI355X (gfx950) brute-force verification engine.
 *
 * Drop-in boundary.  The reference engine (/root/reference/src/brute_force.py) verifies one candidate
 * per OS process: _brute_force() (brute_force.py:106-161) Popen()s one of three verifier executables
 * per password (_call_msoffcrypto_core :163-173, _call_odt_core :175-182, _call_pdf_core :184-197)
 * whose exit code is verify()'s verdict (msoffcrypto_password_verifier.c:52, odt_password_verifier.c:47,
 * pdf_password_verifier.c:60).  This library replaces that inner loop, the three executables and the
 * OpenSSL arithmetic under them with batched gfx950 kernels, one candidate per lane.
 *
 * Plain C types only; no torch or HIP types cross the boundary.  Every call returns DPRF_OK (0) or a
 * negative DPRF_E_* code and sets a thread-local message readable with dprf_last_error().  An error is
 * never reported as "found" (the reference conflates the two: any non-zero exit counts as a hit,
 * brute_force.py:140).
 *
 * Threading: a context spans a list of devices (one or all of the node's GPUs) and owns one host worker
 * thread and one HIP stream per device for the duration of a call: dprf_search_range / dprf_verify_list
 * fan the call out over the devices inside the library (the reference's 4 worker processes on one queue,
 * brute_force.py:70-73 / :92-95, become one worker thread per GPU on one shared chunk cursor).  Calls on
 * DIFFERENT contexts may run concurrently from different threads; calls on the SAME context are
 * serialised by the library (a second caller waits for the first call to return).
 * Every entry point leaves the calling thread's current HIP device as it found it (ABI 5): the library sets the
 * device of each GPU it serves from the calling thread and restores the caller's on return, so a torch user's
 * default device (torch.cuda.current_device()) is not moved by a call (client.py:94-108 treats the verifier as a
 * pure call).
 * Ownership: the caller owns every buffer it passes; they are read/written only during the call.
 */
#ifndef DPRF_H
#define DPRF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPRF_ABI_VERSION 7

/* formats: the tag parse_verification_data extracts (brute_force.py:250) */
#define DPRF_FMT_OFFICE 1   /* "$office$*2007*..."  ECMA-376 Standard Encryption            */
#define DPRF_FMT_ODT 2      /* "$odt$*1.2*..."      ODF 1.2 AES-256-CBC / PBKDF2-HMAC-SHA1     */
#define DPRF_FMT_PDF 3      /* "$pdf$*V*R*..."      PDF standard security handler R2..R6       */

/* error codes */
#define DPRF_OK 0
#define DPRF_E_INVALID (-1)      /* bad argument / malformed field array                          */
#define DPRF_E_DOMAIN (-2)       /* stream outside the parity domain: the reference's behaviour is
                                    undefined or an abort() there           */
#define DPRF_E_HIP (-3)          /* HIP runtime error (message has the hipError string)           */
#define DPRF_E_NODEVICE (-4)     /* no usable gfx950 device / bad device ordinal                  */
#define DPRF_E_PWLEN (-5)        /* candidate too long: over DPRF_MAX_PW bytes (list mode; no argv string can carry
                                    it to the reference), or a range length over DPRF_MAX_PW_RANGE  */
#define DPRF_E_CHARSET (-6)      /* range charset invalid: empty, NUL, a repeated byte, or a byte >= 0x80
                                    for Office (its candidates are UTF-16LE of characters); symbols
                                    (dprf_search_symbols): empty, repeated, with a NUL byte or over 4
                                    bytes, or for Office not one valid UTF-8 character            */

#define DPRF_ALL_DEVICES (-1)    /* dprf_ctx_create device argument: every gfx950 device visible    */
#define DPRF_MAX_DEVICES 64

/* context flags (dprf_ctx_flags) */
#define DPRF_FLAG_NEVER_MATCHES 1        /* reference verify() returns 0 for every candidate: (V,R)
                                            gate / Length%8 (pdf...c:89-101), ev/evh length (office
                                            ...c:163,168).  Searches still run and find nothing.   */
#define DPRF_FLAG_REF_NONDETERMINISTIC 2 /* a hex field starts with 00: the reference's str_to_uchar
                                            (BN_hex2bn/BN_bn2bin) decodes it short and reads
                                            uninitialised bytes; this library decodes it in full.   */

/* List mode takes every candidate the reference's verifiers hash (ABI 5; ABI 4 capped them at a 64-byte slot):
 * ODF and Office any length (odt...c:79 hashes strlen(password); msoffcrypto...c:75,287-296 converts any length to
 * UTF-16LE), PDF R2-R4 truncated at 32 bytes (pdf...c:137), R5 at 127 (:197-206), R6 whole up to DPRF_MAX_PW_R6.
 * Candidates up to 64 bytes after conversion run in 64-byte slots; longer ones go to a long sub-list (k_long_prehash
 * hashes their first message, the format's kernels continue from it) -- same verdicts, same list indices.
 * DPRF_MAX_PW: the reference receives a candidate as one argv string, which Linux caps at MAX_ARG_STRLEN (131,072
 * bytes with the NUL): a longer one never reaches its verifier (DPRF_E_PWLEN).
 * DPRF_MAX_PW_R6: 64 x (pw || K[0:64]) fills the reference's data[(128 + 64 + 48) * 64] (pdf...c:228) at 176 bytes; a
 * longer R6 candidate overflows it and the reference aborts ("stack smashing detected", recorded in
 * tests/golden/long_verdicts.json) -- an error, not a verdict, so DPRF_E_DOMAIN. */
#define DPRF_MAX_PW 131071
#define DPRF_MAX_PW_R6 176
#define DPRF_MAX_PW_RANGE 32   /* longest fixed length for dprf_search_range */

typedef struct dprf_ctx dprf_ctx;

typedef struct dprf_stats {
    uint64_t candidates;   /* candidates fully evaluated on the device                          */
    uint64_t launches;     /* verification-kernel launches                                      */
    double kernel_ms;      /* sum of HIP-event durations of those launches (on the ctx stream)  */
    double wall_ms;        /* host wall time of the call, first launch to last result copy      */
    uint32_t stopped_early;/* 1 if stop_on_first ended the search before the whole range        */
    uint32_t devices;      /* devices that took part in the call (ABI 3; was `reserved`)        */
    double main_kernel_ms; /* HIP-event time of the dominant kernel alone: the KDF kernel for Office/ODF
                              (their check kernel follows it on the same stream), else = kernel_ms  (ABI 2) */
    double hit_ms;         /* host time from the call's start to when the library first knew of a hit, -1 if none
                              (ABI 6): wall_ms - hit_ms is how long the call ran on after its answer existed */
} dprf_stats;
/* kernel_ms / main_kernel_ms are summed over the devices of a multi-device call (device time); wall_ms is
 * the call's wall time.  candidates / launches are totals over the devices.  PDF R2-R4 alternate consecutive
 * launches between two streams per device, so a launch's event time includes the tail of its neighbour on the other
 * stream: their kernel_ms sum can exceed the device time (the library's own chunk sizing times those launches from
 * completion to completion instead). */

/* Per-device record of the last dprf_search_range / dprf_verify_list call on a context (ABI 4): how the shared
 * chunk cursor split the call, so imbalance between devices is visible (the sums above hide it). */
typedef struct dprf_device_stats {
    int32_t device;        /* HIP ordinal                                                              */
    uint32_t launches;     /* chunks this device took                                                  */
    uint64_t candidates;   /* candidates launched on it (before stop_on_first block skips)             */
    double kernel_ms;      /* HIP-event device time of its launches                                    */
    double first_ms;       /* host time from the call's start to its first launch                      */
    double finish_ms;      /* host time from the call's start to when its last launch was retired      */
    uint64_t evaluated;    /* candidates it verified: `candidates` minus the stop_on_first skips (ABI 6) */
} dprf_device_stats;

/* ---- library ---- */
int dprf_abi_version(void);
const char *dprf_last_error(void);
int dprf_device_count(void);      /* gfx950 devices visible to this process */
/* HIP ordinals of the visible gfx950 devices (a non-gfx950 device may sit at any ordinal): writes up to
 * cap ordinals, returns how many there are (ABI 3) */
int dprf_device_list(int *ordinals, int cap);
/* Fingerprint of the sources, Makefile flags and compiler this library was built from (ABI 4): bench.py prints
 * it and tools/prof_summary.py records it, so a profile can be matched to the build it measured. */
const char *dprf_build_id(void);
/* The multi-device chunk policy as a pure function (ABI 4; no device work, usable without a GPU): the size of the
 * next chunk a device of an `ndev`-device call takes from the shared cursor, for the kernel family `kernel`
 * (dprf_ctx_kernel's names), the device's measured rate (candidates per device-ms, 0 = not measured yet), the
 * candidates still unassigned (`remaining`) and the call's size (`total`).  A target-time size (a power of two,
 * ~0.1-3 s of device time by family), capped for ndev > 1 at remaining / (4 ndev) -- guided self-scheduling over
 * the two launches each device keeps in flight, so
 * the chunks shrink as the call runs out and the devices finish together -- but not below the family's tail
 * floor, nor below total / ndev for a call smaller than ndev floors (every device gets a share).  `inflight`: the
 * device's launches still running; with ndev > 1 a device that has one does not take ahead while the remaining
 * work is less than a chunk for every device -- the call returns 0 and the worker first waits for its launch.
 * Returns 0 for an unknown family too. */
uint64_t dprf_plan_chunk(const char *kernel, double rate_per_ms, uint64_t remaining, uint64_t total, int ndev,
                         int inflight);

/* ---- context: one document, one or more devices ----
 * fields/nfields: the array parse_verification_data() returns (brute_force.py:245-264), i.e. the
 * stream split on '*' with fields[0] replaced by the format tag ("office", "odt" or "pdf"); office
 * needs 8 fields, odt 7, pdf 12.  The per-format field meaning is exactly the reference's argv mapping
 * (brute_force.py:163-197).  device: HIP device ordinal, or DPRF_ALL_DEVICES for every gfx950 device. */
int dprf_ctx_create(const char *const *fields, int nfields, int device, dprf_ctx **out);
/* The same over an explicit device list (ABI 3).  An ordinal may repeat: {0,0} runs two streams and two
 * worker threads on device 0 (used to test the multi-device path on one GPU). */
int dprf_ctx_create_devices(const char *const *fields, int nfields, const int *devices, int ndev, dprf_ctx **out);
int dprf_ctx_devices(const dprf_ctx *ctx, int *ordinals, int cap);   /* returns the device count */
int dprf_ctx_destroy(dprf_ctx *ctx);
int dprf_ctx_format(const dprf_ctx *ctx);
int dprf_ctx_flags(const dprf_ctx *ctx);
const char *dprf_ctx_kernel(const dprf_ctx *ctx);   /* kernel family name, e.g. "pdf_r24" */
/* Per-device records of the context's last search / verify call (ABI 4): writes up to cap entries, returns the
 * number of devices of that call (0 before the first call). */
int dprf_ctx_last_call_devices(const dprf_ctx *ctx, dprf_device_stats *out, int cap);

/* ---- range mode: brute_force.py -pr N (init_rangebased_brute_force :60-79, _generate :199-219) ----
 * Verifies candidates [start, start+count) of charset^pwlen in itertools.product order (leftmost
 * character most significant).  The symbols are the charset's BYTES, all distinct (a repeated byte would
 * verify candidates twice: DPRF_E_CHARSET): for PDF and ODF a byte >= 0x80 is a raw candidate byte, as the
 * reference's argv carries it; Office takes ASCII only.  A caller whose alphabet has multi-byte UTF-8
 * characters uses dprf_search_symbols.
 * Writes up to `cap` hit indices, ascending, to hits[]; *nhits = total number of hits found (may exceed cap).
 * stats may be NULL.
 * Multi-device: the devices take contiguous chunks of the range from one shared cursor in increasing
 * order (chunks sized for ~0.1-1 s of device time at the rate measured on that device), so a fast device
 * takes more and every index below the last chunk taken is covered.
 * stop_on_first != 0: the search ends once no unverified index lies below the lowest hit found so far;
 * hits[0] is then the LOWEST verifying index of the whole range, unconditionally (every candidate below
 * it is verified on some device; a kernel block is skipped only if its lowest index is above it).  A
 * multi-device call pushes a hit to the launches already running on the other devices (ABI 6): a host thread
 * polls every lane's host-mapped hit word and publishes the minimum to a word every launch reads beside its own
 * device's (dprf_hits.h), so their blocks above it skip within ~0.2 ms -- as the reference's workers stop at
 * their next candidate once `found` is set (brute_force.py:111-114, :140-147).  The same holds in list mode. */
int dprf_search_range(dprf_ctx *ctx, const uint8_t *charset, int cslen, int pwlen, uint64_t start,
                      uint64_t count, int stop_on_first, uint64_t *hits, int64_t cap, int64_t *nhits,
                      dprf_stats *stats);

/* ---- range mode over multi-byte symbols (ABI 7): a --charset with non-ASCII characters ----
 * Verifies indices [start, start+count) of sym^pwlen in itertools.product order over SYMBOLS (the last position
 * fastest, brute_force.py:205), symbol k being the bytes sym[sym_off[k] .. sym_off[k+1]) -- a charset's characters
 * in UTF-8, each 1-4 bytes, all distinct, no NUL byte (DPRF_E_CHARSET).  For Office each symbol must be one valid
 * UTF-8 character and goes in as its UTF-16LE, as iconv converts the whole password (msoffcrypto...c:275-336).  The
 * device spells every candidate into a list slot and the list-mode kernels verify it: a candidate's bytes are the
 * concatenation of its symbols' (PDF R2-R4 hash the first 32, pdf...c:137).  DPRF_E_PWLEN: pwlen outside
 * 1..DPRF_MAX_PW_RANGE, or a candidate could exceed a 64-byte slot after conversion and truncation (the caller
 * spells such windows itself and uses dprf_verify_list).  hits[] are indices relative to `start`; the rest is as
 * dprf_search_range (stop_on_first, multi-device chunks and the cross-device stop). */
int dprf_search_symbols(dprf_ctx *ctx, const uint8_t *sym, const uint32_t *sym_off, int nsym, int pwlen,
                        uint64_t start, uint64_t count, int stop_on_first, uint64_t *hits, int64_t cap,
                        int64_t *nhits, dprf_stats *stats);

/* ---- list mode: client payloads (init_listbased_brute_force :82-104, client.py:105) ----
 * Candidate k is blob[offsets[k] .. offsets[k+1]) (n+1 offsets).  Hits are list indices. */
int dprf_verify_list(dprf_ctx *ctx, const uint8_t *blob, const uint64_t *offsets, int64_t n,
                     int stop_on_first, uint64_t *hits, int64_t cap, int64_t *nhits, dprf_stats *stats);
/* dprf_verify_list rejects the whole call if one candidate is one the reference cannot verify (NUL; empty or
 * invalid-UTF-8 Office password; PDF R6 over DPRF_MAX_PW_R6 bytes: DPRF_E_DOMAIN / DPRF_E_INVALID; over DPRF_MAX_PW
 * bytes: DPRF_E_PWLEN).  This host-only check (no
 * device work) writes 0 or that DPRF_E_* code per candidate to status[n] (may be NULL) and returns the
 * number of invalid candidates, so a caller can drop them and verify the rest -- the reference fails
 * such a candidate alone, in its own verifier process (brute_force.py:163-197).  (ABI 3) */
int dprf_list_status(const dprf_ctx *ctx, const uint8_t *blob, const uint64_t *offsets, int64_t n, int8_t *status);

#ifdef __cplusplus
}
#endif
#endif
