// dev_slots.hpp — job descriptors: the port table, its bit rows and the per-(slot, word) descriptor words.
// Part of engine.hip's single translation unit (device bodies inline across stages, host helpers are
// static): included once, by engine.hip, in stage order.
#pragma once

namespace cyc {

// PortMatcher.Allows(ResolvedPort, ResolvedPortName, Protocol) — portmatcher.go:10-92, 190-199.
__device__ __forceinline__ void portok_blk(uint32_t M, uint32_t D, const DPortM* pms, const DPortEntry* pents, const DDesc* descs,
                         uint8_t* __restrict__ portok, uint32_t bid_, uint32_t nblk_) {
  uint32_t i = bid_ * blockDim.x + threadIdx.x;
  if (i >= M * D) return;
  uint32_t m = i / D, e = i % D;
  DPortM pm = pms[m];
  DDesc d = descs[e];
  uint8_t ok = pm.all ? 1 : 0;
  for (uint32_t j = 0; j < pm.ecnt && !ok; j++) {
    DPortEntry pe = pents[pm.eoff + j];
    if (pe.proto != d.proto) continue;  // raw protocol string compare ("tcp" != "TCP")
    switch (pe.kind) {
      case PE_PROTO: ok = 1; break;
      case PE_INT: ok = pe.a == d.port; break;
      case PE_NAME: ok = uint32_t(pe.a) == d.name; break;
      default: ok = pe.a <= d.port && d.port <= pe.b; break;
    }
  }
  portok[i] = ok;
}
__global__ void k_portok(uint32_t M, uint32_t D, const DPortM* pms, const DPortEntry* pents, const DDesc* descs,
                         uint8_t* __restrict__ portok) { portok_blk(M, D, pms, pents, descs, portok, blockIdx.x, gridDim.x); }

// Port table rows as descriptor bit masks (D <= 32): the egress class rows test a peer's port
// matcher against a per-word descriptor with a shift of one block-uniform word instead of a
// vector byte load per (slot, peer).
__device__ __forceinline__ void portbits_blk(uint32_t M, uint32_t D, const uint8_t* __restrict__ portok,
                                             uint32_t* __restrict__ portbits, uint32_t bid_) {
  const uint32_t m = bid_ * 256 + threadIdx.x;
  if (m >= M) return;
  uint32_t bits = 0;
  for (uint32_t e = 0; e < D; e++) bits |= portok[uint64_t(m) * D + e] ? (1u << e) : 0u;
  portbits[m] = bits;
}
// The same bit rows straight from the port matchers (no byte table first): launch B builds them next
// to the byte table when there is no launch A, so the identity sets of launch D can read them.
__device__ __forceinline__ void portbits_direct_blk(uint32_t M, uint32_t D, const DPortM* pms, const DPortEntry* pents,
                                                    const DDesc* descs, uint32_t* __restrict__ portbits, uint32_t bid_) {
  const uint32_t m = bid_ * 256 + threadIdx.x;
  if (m >= M) return;
  const DPortM pm = pms[m];
  uint32_t bits = pm.all ? (D >= 32 ? ~0u : (1u << D) - 1u) : 0u;
  // the matcher's entries PB_ENT at a time, all loaded before any test (one memory round trip per
  // batch, not one per (descriptor, entry)), each tested against every descriptor (block-uniform
  // loads): launch B config #3 81.4 -> 79.9 us, its N = 8 source shard 33 -> 26.5 us (the port bits
  // were that shard's longest chain); 4 at a time: the same times at +5 VGPRs for all of launch B
  // (profiles/r04_front_b_ab.txt)
  constexpr uint32_t PB_ENT = 2;
  for (uint32_t j0 = 0; !pm.all && j0 < pm.ecnt; j0 += PB_ENT) {
    DPortEntry pe[PB_ENT];
#pragma unroll
    for (uint32_t x = 0; x < PB_ENT; x++) pe[x] = pents[pm.eoff + min(j0 + x, pm.ecnt - 1)];
    for (uint32_t e = 0; e < D; e++) {
      const DDesc d = descs[e];
      bool ok = false;
#pragma unroll
      for (uint32_t x = 0; x < PB_ENT; x++)  // raw protocol string compare ("tcp" != "TCP")
        ok = ok || (pe[x].proto == d.proto &&
                    (pe[x].kind == PE_PROTO ? true
                     : pe[x].kind == PE_INT ? pe[x].a == d.port
                     : pe[x].kind == PE_NAME ? uint32_t(pe[x].a) == d.name
                                             : pe[x].a <= d.port && d.port <= pe[x].b));
      bits |= ok ? 1u << e : 0u;
    }
  }
  portbits[m] = bits;
}
__global__ __launch_bounds__(256) void k_portbits(uint32_t M, uint32_t D, const uint8_t* __restrict__ portok,
                                                  uint32_t* __restrict__ portbits) {
  portbits_blk(M, D, portok, portbits, blockIdx.x);
}

// Per (slot k, word w over pods-as-destinations): VALID bits, the word's common descriptor
// (DESCW >= 0), none valid (-2) or mixed (-1), and per-descriptor masks DM for mixed words.
__device__ __forceinline__ void slot_words_blk(uint32_t P, uint32_t K, uint32_t W, uint32_t D,
                                                    const int32_t* __restrict__ slot_desc,
                                                    const uint8_t* __restrict__ slot_status, uint64_t* __restrict__ VALID,
                                                    int32_t* __restrict__ DESCW, uint64_t* __restrict__ DM, uint32_t bid_, uint32_t nblk_) {
  uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t idx = __builtin_amdgcn_readfirstlane(bid_ * 4 + wave);  // (k, w), wave-uniform
  if (idx >= K * W) return;
  uint32_t k = idx / W, w = idx % W;
  uint32_t q = w * 64 + lane;
  int32_t e = -1;
  bool valid = false;
  if (q < P) {
    valid = slot_status[uint64_t(q) * K + k] == CYC_JOB_VALID;
    e = valid ? slot_desc[uint64_t(q) * K + k] : -1;
  }
  uint64_t vm = __ballot(valid);
  // first valid lane's descriptor, broadcast
  int32_t first = -2;
  if (vm) first = __shfl(e, __ffsll((unsigned long long)vm) - 1);
  bool same = !valid || e == first;
  uint64_t sm = __ballot(same);
  int32_t dw = vm == 0 ? -2 : (sm == ~0ull ? first : -1);
  if (lane == 0) {
    VALID[uint64_t(k) * W + w] = vm;
    DESCW[uint64_t(k) * W + w] = dw;
  }
  if (dw == -1) {
    for (uint32_t d = 0; d < D; d++) {
      uint64_t m = __ballot(valid && e == int32_t(d));
      if (lane == 0) DM[(uint64_t(k) * D + d) * W + w] = m;
    }
  }
}
__global__ __launch_bounds__(256) void k_slot_words(uint32_t P, uint32_t K, uint32_t W, uint32_t D,
                                                    const int32_t* __restrict__ slot_desc,
                                                    const uint8_t* __restrict__ slot_status, uint64_t* __restrict__ VALID,
                                                    int32_t* __restrict__ DESCW, uint64_t* __restrict__ DM) { slot_words_blk(P, K, W, D, slot_desc, slot_status, VALID, DESCW, DM, blockIdx.x, gridDim.x); }

}  // namespace cyc
