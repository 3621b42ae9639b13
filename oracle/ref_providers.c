/* Test infrastructure (oracle/): activates OpenSSL 3's default + legacy providers in-process so the
 * reference PDF verifier's EVP_rc4()/EVP_rc4_40() calls (pdf_password_verifier.c:445-453) work when
 * the reference verify() is called from the CPU-baseline harness.  Not part of the product. */
#include <openssl/provider.h>

int ref_load_legacy(void) {
    OSSL_PROVIDER *d = OSSL_PROVIDER_load(NULL, "default");
    OSSL_PROVIDER *l = OSSL_PROVIDER_load(NULL, "legacy");
    return (d != NULL) && (l != NULL);
}
