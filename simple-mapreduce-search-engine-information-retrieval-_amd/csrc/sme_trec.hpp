// sme_trec.hpp -- TrecDocument.getDocid on a record's raw bytes
// (C/edu/umd/cloud9/collection/trec/TrecDocument.java:76-89).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sme {

// indexOf("<DOCNO>"), then indexOf("</DOCNO>", start), then trim().  Returns
// false when "<DOCNO>" has no "</DOCNO>" after it (substring(start + 7, -1)
// throws: the map task fails).  No "<DOCNO>": docid "" ([*ib, *ie) empty).
// Trimming bytes <= 0x20 equals String.trim() on the decoded string: units
// <= U+0020 are exactly those single bytes.
__device__ __forceinline__ bool docid_span(const uint8_t *t, int64_t s, int64_t e, int64_t *ib, int64_t *ie) {
  int64_t a = -1;
  for (int64_t p = s; p + 7 <= e; p++) {
    if (t[p] == '<' && t[p + 1] == 'D' && t[p + 2] == 'O' && t[p + 3] == 'C' && t[p + 4] == 'N' &&
        t[p + 5] == 'O' && t[p + 6] == '>') {
      a = p;
      break;
    }
  }
  if (a < 0) {
    *ib = *ie = 0;
    return true;
  }
  int64_t z = -1;
  for (int64_t p = a; p + 8 <= e; p++) {
    if (t[p] == '<' && t[p + 1] == '/' && t[p + 2] == 'D' && t[p + 3] == 'O' && t[p + 4] == 'C' &&
        t[p + 5] == 'N' && t[p + 6] == 'O' && t[p + 7] == '>') {
      z = p;
      break;
    }
  }
  if (z < 0) return false;
  int64_t b = a + 7, f = z;
  while (b < f && t[b] <= 0x20) b++;
  while (f > b && t[f - 1] <= 0x20) f--;
  *ib = b;
  *ie = f;
  return true;
}

}  // namespace sme
