// Per-lane verdict statuses — the data half of the C-ABI contract
// (include/cordahip.h CORDAHIP_STATUS_*). Mapping to the reference's
// exceptions: SURVEY.md §8(b) "Per-lane status -> Kotlin semantics".
#pragma once
#include <stdint.h>

namespace cordahip {
static constexpr uint8_t kStatusOk = 0;           // isValid true / doVerify true
static constexpr uint8_t kStatusBadSig = 1;       // isValid false / doVerify SignatureException
static constexpr uint8_t kStatusMalformedSig = 2; // engine SignatureException
static constexpr uint8_t kStatusBadKey = 3;       // key decode IllegalArgumentException
static constexpr uint8_t kStatusUnsupported = 4;  // IllegalArgumentException (scheme)
static constexpr uint8_t kStatusEmpty = 5;        // IllegalArgumentException (empty input)
}  // namespace cordahip
