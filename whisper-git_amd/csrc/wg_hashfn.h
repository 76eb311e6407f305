// wg_hashfn.h — 20-byte commit-id keys for the HBM hash tables
// (wg_hash.hip, wg_shard.hip): open addressing, 8-byte entries
// {fingerprint:32 | row:32}, full-key compare against the id array.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {

constexpr uint64_t HEMPTY = ~0ull;

struct Key { uint32_t w[5]; };

__device__ __forceinline__ Key load_key(const uint8_t *p) {
    // ids are 20-byte records in hipMalloc'd arrays: 4-byte aligned
    const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
    Key k;
#pragma unroll
    for (int i = 0; i < 5; i++) k.w[i] = q[i];
    return k;
}
__device__ __forceinline__ bool key_eq(const Key &a, const uint8_t *p) {
    const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
    return a.w[0] == q[0] && a.w[1] == q[1] && a.w[2] == q[2] && a.w[3] == q[3] && a.w[4] == q[4];
}
__device__ __forceinline__ uint64_t key_hash(const Key &k) {
    uint64_t h = ((uint64_t)k.w[1] << 32 | k.w[0]) ^ ((uint64_t)k.w[3] * 0x9E3779B97F4A7C15ull) ^ k.w[4];
    h ^= h >> 31; h *= 0x7FB5D329728EA185ull; h ^= h >> 27; h *= 0x81DADEF4BC2DD44Dull; h ^= h >> 33;
    return h;
}
__device__ __forceinline__ uint32_t key_fp(const Key &k) { return k.w[2] ^ (k.w[4] * 0x85EBCA6Bu); }

__device__ __forceinline__ int64_t hash_find(const Key &k, const uint8_t *__restrict__ oid,
                                             const unsigned long long *__restrict__ table, uint64_t mask) {
    const uint32_t fp = key_fp(k);
    uint64_t h = key_hash(k) & mask;
    for (uint64_t probes = 0; probes <= mask; probes++) {
        const unsigned long long cur = table[h];
        if (cur == HEMPTY) return -1;
        if ((uint32_t)(cur >> 32) == fp && key_eq(k, oid + (uint64_t)(uint32_t)cur * 20)) return (int64_t)(uint32_t)cur;
        h = (h + 1) & mask;
    }
    return -1;
}

}  // namespace
