// sst_pyset.h -- the iteration order of CPython's set, restated for the
// skeleton walk (host and device).
//
// SkeletonBuilder's results depend on Python set iteration order
// (skeleton_building.py:442-482: `for p in pos` over a set of ints, and the
// explanation lists, which calculate_explanations builds by iterating a set
// of name tuples, common.py:60-65 / mass_explanation.py:287-320, grouped by
// length with itertools.groupby).  The order is a pure function of the
// elements' hashes and the insertion sequence, so it is emulated here
// exactly: Objects/setobject.c (CPython 3.7-3.12: set_add_entry with
// LINEAR_PROBES = 9 and PERTURB_SHIFT = 5, set_table_resize to the smallest
// power of two above used * 4 once fill * 5 >= mask * 3, re-insertion of the
// old table in slot order by set_insert_clean) and Objects/tupleobject.c
// (tuplehash, the xxHash-style combiner of 3.8+).  Element hashes come from
// the caller: an int hashes to itself (the small non-negative positions), a
// name tuple from the names' str hashes, which the host takes from the
// running interpreter (hash(name): PYTHONHASHSEED applies as in the
// reference).  No element is ever removed (the walk's sets only grow), so
// the tables hold no dummies.  tests/test_pyset.py checks both against the
// interpreter on random sets.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SST_HD __host__ __device__ __forceinline__
#else
#define SST_HD inline
#endif

namespace sst {
namespace pyset {

constexpr int kLinearProbes = 9;
constexpr int kPerturbShift = 5;
constexpr uint32_t kMinSize = 8;  // PySet_MINSIZE

// tuplehash (64-bit Py_uhash_t)
SST_HD int64_t tuple_hash_step(uint64_t acc, int64_t item) {
  const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull;
  acc += (uint64_t)item * P2;
  acc = (acc << 31) | (acc >> 33);
  acc *= P1;
  return (int64_t)acc;
}
SST_HD uint64_t tuple_hash_init() { return 2870177450012600261ull; }  // _PyHASH_XXPRIME_5
SST_HD int64_t tuple_hash_final(uint64_t acc, int64_t len) {
  acc += (uint64_t)len ^ (2870177450012600261ull ^ 3527539ull);
  if (acc == ~0ull) return 1546275796;
  return (int64_t)acc;
}

// table size after `n` distinct insertions into an empty set (no removals)
SST_HD uint32_t table_size_for(uint32_t n) {
  uint32_t mask = kMinSize - 1, fill = 0;
  for (uint32_t k = 0; k < n; ++k) {
    ++fill;
    if ((uint64_t)fill * 5 >= (uint64_t)mask * 3) {
      const uint64_t minused = fill > 50000 ? (uint64_t)fill * 2 : (uint64_t)fill * 4;
      uint64_t size = kMinSize;
      while (size <= minused) size <<= 1;
      mask = (uint32_t)size - 1;
    }
  }
  return mask + 1;
}

// A set over caller storage: slots [0, cap) of `key` (-1 empty) and `hash`,
// plus a second pair of arrays of the same capacity for resizes (the table
// alternates between the two).  Keys identify elements (equal keys = equal
// elements); hashes are the elements' Python hashes.
struct Table {
  int32_t* key[2];
  int64_t* hash[2];
  uint32_t cap;   // slots per array (a power of two >= the largest table)
  uint32_t mask;  // current table size - 1
  uint32_t fill;
  int cur;        // which array holds the table
  bool overflow;  // the table outgrew `cap`: its order is unknown
};

SST_HD void clear(Table& t) {
  t.mask = kMinSize - 1;
  t.fill = 0;
  t.cur = 0;
  t.overflow = t.cap < kMinSize;
  if (t.overflow) return;
  for (uint32_t i = 0; i < kMinSize; ++i) t.key[0][i] = -1;
}

// set_insert_clean: the first empty slot on the probe sequence
SST_HD void insert_clean(int32_t* key, int64_t* hash, uint32_t mask, int32_t k, int64_t h) {
  uint64_t perturb = (uint64_t)h;
  uint32_t i = (uint32_t)((uint64_t)h & mask);
  for (;;) {
    if (key[i] < 0) {
      key[i] = k;
      hash[i] = h;
      return;
    }
    if (i + kLinearProbes <= mask) {
      for (int j = 1; j <= kLinearProbes; ++j) {
        if (key[i + j] < 0) {
          key[i + j] = k;
          hash[i + j] = h;
          return;
        }
      }
    }
    perturb >>= kPerturbShift;
    i = (uint32_t)((i * 5ull + 1 + perturb) & mask);
  }
}

// set_add_entry; returns false when the element was already present
SST_HD bool add(Table& t, int32_t k, int64_t h) {
  if (t.overflow) return false;
  int32_t* key = t.key[t.cur];
  int64_t* hash = t.hash[t.cur];
  const uint32_t mask = t.mask;
  uint64_t perturb = (uint64_t)h;
  uint32_t i = (uint32_t)((uint64_t)h & mask);
  int32_t slot = -1;
  for (;;) {
    const int probes = (i + kLinearProbes <= mask) ? kLinearProbes : 0;
    for (int j = 0; j <= probes; ++j) {
      const uint32_t s = i + (uint32_t)j;
      if (key[s] < 0) {
        slot = (int32_t)s;
        break;
      }
      if (hash[s] == h && key[s] == k) return false;  // found_active
    }
    if (slot >= 0) break;
    perturb >>= kPerturbShift;
    i = (uint32_t)((i * 5ull + 1 + perturb) & mask);
  }
  key[slot] = k;
  hash[slot] = h;
  ++t.fill;
  if ((uint64_t)t.fill * 5 < (uint64_t)mask * 3) return true;
  // set_table_resize(so, used > 50000 ? used * 2 : used * 4)
  const uint64_t minused = t.fill > 50000 ? (uint64_t)t.fill * 2 : (uint64_t)t.fill * 4;
  uint64_t size = kMinSize;
  while (size <= minused) size <<= 1;
  if (size > t.cap) {
    t.overflow = true;
    return true;
  }
  const int nxt = t.cur ^ 1;
  int32_t* nkey = t.key[nxt];
  int64_t* nhash = t.hash[nxt];
  const uint32_t nmask = (uint32_t)size - 1;
  for (uint32_t s = 0; s <= nmask; ++s) nkey[s] = -1;
  for (uint32_t s = 0; s <= mask; ++s)
    if (key[s] >= 0) insert_clean(nkey, nhash, nmask, key[s], hash[s]);
  t.cur = nxt;
  t.mask = nmask;
  return true;
}

}  // namespace pyset
}  // namespace sst
