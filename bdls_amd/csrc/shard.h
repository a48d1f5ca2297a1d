// In-process multi-device split of one host batch (bh_verify / bh_verify_submit
// over every initialised device, bdls_hip.cpp submit_job): contiguous shards
// of [0, n), each starting at a multiple of 64 records, so a shard's bitmap
// begins on a byte (and u64 word) boundary of the caller's bitmap and the
// shards' result bytes never share a byte. The last shard is ragged. Pure host
// code: tests/native/hostsim.cpp checks the arithmetic and the bitmap merge.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>

namespace bh {

struct Shard {
  size_t lo, len;
};

// Devices that get work: at most one per 64 records.
inline size_t shard_devices(size_t n, size_t ndev) {
  const size_t groups = (n + 63) / 64;
  return ndev < groups ? ndev : groups;
}

// Shard k of [0, n) over ndev devices: the ceil(n / 64) groups of 64 records
// dealt out in contiguous, balanced runs (every device that gets work gets at
// least one group; the last shard ends at n).
inline Shard shard_of(size_t n, size_t ndev, size_t k) {
  const size_t nd = shard_devices(n, ndev), groups = (n + 63) / 64;
  if (k >= nd) return Shard{n, 0};
  const size_t glo = k * groups / nd, ghi = (k + 1) * groups / nd;
  const size_t lo = 64 * glo, hi = 64 * ghi < n ? 64 * ghi : n;
  return Shard{lo, hi - lo};
}

// A shard's results into the caller's LSB-first bitmap: its bitmap words
// (bit i = record lo + i) start at byte lo / 8.
inline void shard_bitmap_merge(uint8_t* bitmap, const Shard& s, const void* words) {
  if (s.len) std::memcpy(bitmap + s.lo / 8, words, (s.len + 7) / 8);
}

}  // namespace bh
