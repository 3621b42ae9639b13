/* dprf_launch.h -- host-side launchers of the verification kernels (internal to libdprf.so). */
#ifndef DPRF_LAUNCH_H
#define DPRF_LAUNCH_H
#include <hip/hip_runtime.h>
#include "dprf_params.h"

/* keys: device scratch of >= 8 * e.count words (the derived keys handed from the KDF to the check kernel);
 * mid: if non-null, recorded on s between the KDF kernel and the check kernel (dominant-kernel timing) */
hipError_t launch_office(const dprf_enum &e, const dprf_office_params &p, const dprf_aes_tables *T,
                         dprf_results *R, uint32_t cap, uint32_t stop, hipStream_t s, uint32_t *keys,
                         hipEvent_t mid);
hipError_t launch_odt(const dprf_enum &e, const dprf_odt_params &p, const dprf_aes_tables *T,
                      dprf_results *R, uint32_t cap, uint32_t stop, hipStream_t s, uint32_t *keys,
                         hipEvent_t mid);
hipError_t launch_pdf_r5(const dprf_enum &e, const dprf_pdf_params &p, dprf_results *R, uint32_t cap,
                         uint32_t stop, hipStream_t s);
hipError_t launch_pdf_r24(const dprf_enum &e, const dprf_pdf_params &p, dprf_results *R, uint32_t cap,
                          uint32_t stop, hipStream_t s);
/* long list (e.mode 2): the records' first-message hash into e.keys, or (DPRF_LONG_R5) the whole R5 check */
hipError_t launch_long_prehash(const dprf_enum &e, const dprf_long_params &lp, dprf_results *R, uint32_t cap,
                               uint32_t stop, hipStream_t s);
/* symbol windows (dprf_search_symbols): e.count candidates from the digits in e.sdig (base e.cslen), symbol table
 * symtab = [256] LE-packed bytes + [256] byte counts, into slots[n][DPRF_SLOT_WORDS] / lens[n]; bytes at or past
 * trunc stay zero */
hipError_t launch_spell_symbols(const dprf_enum &e, const uint32_t *symtab, uint32_t trunc, uint32_t *slots,
                                uint8_t *lens, hipStream_t s);
hipError_t launch_pdf_r6(const dprf_enum &e, const dprf_pdf_params &p, const dprf_aes_tables *T,
                         dprf_results *R, uint32_t cap, uint32_t stop, hipStream_t s);
#endif
