/*
 * ref_hash_shim.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Thin ctypes-friendly harness around the reference's own AVL interval index
 * (/root/reference/tools/hash.c, compiled unchanged from where it lies by
 * oracle/Makefile into oracle/_ref/libref_hash.so).  It lets the tests check
 * the oracle's and the engine's flattened lookup (sorted unique keys + LIFO
 * entry lists) against the real ht_insert / ht_lower_key / FOREACH_HASH
 * (tools/hash.c:63-77, 108-114, 204-231; tools/hash.h:75-78).
 *
 * Values stored in the tree are entry ids (1-based, cast to pointers).
 */
#include <stdint.h>
#include <stdlib.h>
#include "hash.h"

static struct ht_node *root = NULL;

void ref_reset(void) {
  if (root) ht_release(root);
  root = NULL;
}

/* insert (key, id) in insertion (allocation) order, as ht_insert does for
 * every ma_record_malloc / insert_memory_info / stack registration */
void ref_insert(uint64_t key, uint64_t id) { root = ht_insert(root, key, (void *)(uintptr_t)id); }

/* ht_lower_key(addr): writes the node key and up to `cap` entry ids in list
 * order (newest first); returns the number of entries, or -1 if no node. */
int ref_lower_key(uint64_t addr, uint64_t *key_out, uint64_t *ids, int cap) {
  struct ht_node *n = ht_lower_key(root, addr);
  if (!n) return -1;
  *key_out = n->key;
  int k = 0;
  for (struct ht_entry *e = n->entries; e; e = e->next) {
    if (k < cap) ids[k] = (uint64_t)(uintptr_t)e->value;
    k++;
  }
  return k;
}

/* FOREACH_HASH order: writes (key, id) pairs; returns the count */
int64_t ref_foreach(uint64_t *keys, uint64_t *ids, int64_t cap) {
  int64_t k = 0;
  struct ht_node *n = NULL;
  FOREACH_HASH(root, n) {
    for (struct ht_entry *e = n->entries; e; e = e->next) {
      if (k < cap) {
        keys[k] = n->key;
        ids[k] = (uint64_t)(uintptr_t)e->value;
      }
      k++;
    }
  }
  return k;
}

int ref_size(void) { return ht_size(root); }
void ref_check(void) { ht_check(root); }
