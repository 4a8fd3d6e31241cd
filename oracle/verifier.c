/* ORACLE — test infrastructure only.  Verifier: see below (filled in later). */
#include "oracle.h"
int orc_verify_segment(const uint8_t *proof, size_t len, const zkl_air_public_inputs *pi,
                       const zkl_proof_options *opts, char *err, size_t errlen) {
  (void)proof; (void)len; (void)pi; (void)opts; (void)err; (void)errlen;
  return -1;
}
