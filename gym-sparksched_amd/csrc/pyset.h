// pyset.h — CPython 3.10 `set` model for small non-negative int keys (executor ids).
//
// The reference picks executors by set iteration order: set.pop() in _fulfill_commitments_from_source
// (spark_sched_sim.py:730-743) and list(set) in _move_idle_executors (:745-782), over sets built from
// ExecutorTracker pools (executor_tracker.py:32-70, 186-220) that see add/remove churn. Order depends on
// the full table history, so each pool keeps an emulated table:
//   probe: i = h & mask; slot i, then the 9 following slots only if i + 9 <= mask; then
//          perturb >>= 5; i = (i*5 + 1 + perturb) & mask            (hash(int) = int)
//   add:   key found -> no-op; first EMPTY ends the probe: reuse the LAST dummy seen, else take the
//          empty slot (fill++), resizing to the smallest power of two > used*4 once fill*5 >= mask*3
//   remove: slot -> DUMMY (no resize);  iteration/pop order = table order.
// Pinned against CPython by tests/test_kats.py (random add/remove/copy/set(gen)/pop traces).
#pragma once
#include <stdint.h>

namespace ssim {

constexpr uint8_t kSlotEmpty = 0xFF;
constexpr uint8_t kSlotDummy = 0xFE;

// table metadata of one set (layout.h keeps pools' metadata in the hot block, 6 bytes each)
struct PySetMeta {
  uint16_t mask, fill, used;
};
static_assert(sizeof(PySetMeta) == 6, "pool metadata is 6 bytes in the hot block");

// Execution: every lane of the wave runs these with identical (wave-uniform) keys and tables; each
// table / metadata read goes through W::uni so the probe loops are scalar code, and writes are
// same-address stores from all lanes (one LDS access). The 1-lane host build runs the same code.
__device__ __forceinline__ void ps_init(PySetMeta* m, uint8_t* tab) {
  m->mask = 7;
  m->fill = 0;
  m->used = 0;
  for (int i = 0; i < 8; ++i) tab[i] = kSlotEmpty;
}

// set_insert_clean: table known to contain no dummies and not `key`.
template <class W>
__device__ __forceinline__ void ps_insert_clean(uint8_t* tab, uint32_t mask, uint32_t key) {
  uint32_t i = key & mask, perturb = key;
  for (;;) {
    if (W::uni(tab[i]) == kSlotEmpty) {
      tab[i] = (uint8_t)key;
      return;
    }
    if (i + 9u <= mask) {
      for (uint32_t j = 1; j <= 9u; ++j) {
        if (W::uni(tab[i + j]) == kSlotEmpty) {
          tab[i + j] = (uint8_t)key;
          return;
        }
      }
    }
    perturb >>= 5;
    i = (i * 5u + 1u + perturb) & mask;
  }
}

// Active keys in table order (= iteration order = pop order of a fresh set). Returns the count.
template <class W>
__device__ __forceinline__ int ps_keys(const PySetMeta* m, const uint8_t* tab, int32_t* out) {
  int n = 0;
  const int size = (int)W::uni(m->mask) + 1;
  for (int i = 0; i < size; ++i) {
    const uint8_t v = W::uni(tab[i]);
    if (v < kSlotDummy) out[n++] = v;
  }
  return n;
}

// set_table_resize(so, minused): clean re-insert of the active keys (old table order).
template <class W>
__device__ __forceinline__ void ps_resize(PySetMeta* m, uint8_t* tab, int minused, int32_t* tmp) {
  const int n = ps_keys<W>(m, tab, tmp);
  uint32_t size = 8;
  while ((int)size <= minused) size <<= 1;
  for (uint32_t i = 0; i < size; ++i) tab[i] = kSlotEmpty;
  const uint32_t mask = size - 1;
  for (int k = 0; k < n; ++k) ps_insert_clean<W>(tab, mask, (uint32_t)W::uni(tmp[k]));
  m->mask = (uint16_t)mask;
  m->fill = (uint16_t)n;
  m->used = (uint16_t)n;
}

// set_add_entry for an int key. `tmp` needs room for used+1 keys (resize scratch).
template <class W>
__device__ __forceinline__ void ps_add(PySetMeta* m, uint8_t* tab, uint32_t key, int32_t* tmp) {
  const uint32_t mask = W::uni(m->mask);
  const uint32_t fill = W::uni(m->fill), used = W::uni(m->used);
  uint32_t i = key & mask, perturb = key;
  int freeslot = -1;
  for (;;) {
    const uint32_t probes = (i + 9u <= mask) ? 9u : 0u;
    for (uint32_t j = 0; j <= probes; ++j) {
      const uint32_t idx = i + j;
      const uint8_t v = W::uni(tab[idx]);
      if (v == kSlotEmpty) {
        if (freeslot >= 0) {
          tab[freeslot] = (uint8_t)key;
          m->used = (uint16_t)(used + 1);
          return;
        }
        tab[idx] = (uint8_t)key;
        m->fill = (uint16_t)(fill + 1);
        m->used = (uint16_t)(used + 1);
        if ((fill + 1) * 5u >= mask * 3u) ps_resize<W>(m, tab, (int)(used + 1) * 4, tmp);
        return;
      }
      if (v == key) return;
      if (v == kSlotDummy) freeslot = (int)idx;
    }
    perturb >>= 5;
    i = (i * 5u + 1u + perturb) & mask;
  }
}

// set.remove(key) via set_lookkey's probe sequence. Returns false if absent (KeyError in CPython).
template <class W>
__device__ __forceinline__ bool ps_remove(PySetMeta* m, uint8_t* tab, uint32_t key) {
  const uint32_t mask = W::uni(m->mask);
  uint32_t i = key & mask, perturb = key;
  for (;;) {
    const uint32_t probes = (i + 9u <= mask) ? 9u : 0u;
    for (uint32_t j = 0; j <= probes; ++j) {
      const uint8_t v = W::uni(tab[i + j]);
      if (v == kSlotEmpty) return false;
      if (v == key) {
        tab[i + j] = kSlotDummy;
        m->used = (uint16_t)(W::uni(m->used) - 1);
        return true;
      }
    }
    perturb >>= 5;
    i = (i * 5u + 1u + perturb) & mask;
  }
}

// Iteration order of `src.copy()` (set_merge into a fresh set: one pre-resize to > used*2 when
// used*5 >= 21, then slot copy if same mask and no dummies, else clean insert in source order).
// `keys` holds src's keys in table order on entry (n of them) and the copy's order on exit.
template <class W>
__device__ __forceinline__ void ps_copy_order(const PySetMeta* src, int32_t* keys, int n, uint8_t* tab) {
  if (n == 0) return;
  uint32_t size = 8;
  if (n * 5 >= 21) {
    while ((int)size <= n * 2) size <<= 1;
  }
  const uint32_t mask = size - 1;
  if (mask == W::uni(src->mask) && W::uni(src->fill) == W::uni(src->used)) return;  // slot copy keeps order
  for (uint32_t i = 0; i < size; ++i) tab[i] = kSlotEmpty;
  for (int k = 0; k < n; ++k) ps_insert_clean<W>(tab, mask, (uint32_t)W::uni(keys[k]));
  int c = 0;
  for (uint32_t i = 0; i < size; ++i) {
    const uint8_t v = W::uni(tab[i]);
    if (v != kSlotEmpty) keys[c++] = v;
  }
}

// Table order of `set(keys)` built by sequential adds into a fresh set (no removals, so no dummies).
// In-place on `keys` (n entries); `tab` and `tmp` are scratch.
template <class W>
__device__ __forceinline__ void ps_build_order(int32_t* keys, int n, uint8_t* tab, int32_t* tmp) {
  PySetMeta m;
  ps_init(&m, tab);
  for (int k = 0; k < n; ++k) ps_add<W>(&m, tab, (uint32_t)W::uni(keys[k]), tmp);
  ps_keys<W>(&m, tab, keys);
}

}  // namespace ssim
