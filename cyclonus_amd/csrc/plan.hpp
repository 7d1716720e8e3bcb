// plan.hpp — the run planner: identities, peer plans, device tables, range plans.
// Part of engine.hip's single translation unit (device bodies inline across stages, host helpers are
// static): included once, by engine.hip, in stage order.
#pragma once

// Pod identities per direction, numbered by first appearance in pod order: egress (namespace, label
// set), ingress (namespace, label set, every slot's job status and descriptor).  Hashed into an
// open-addressing table whose entries hold their first pod; a probe compares the pods' fields.
static void build_identities(cyc_ctx* c) {
  Problem& pb = c->pb;
  const uint32_t K = pb.K;
  uint32_t cap = 2;
  while (cap < 2 * std::max<uint32_t>(pb.P, 1)) cap <<= 1;
  std::vector<uint32_t> slot_pod(cap), slot_id(cap);
  for (int d = 0; d < 2; d++) {
    Identities& I = c->ids[d];
    I = Identities{};
    I.of_pod.resize(pb.P);
    const bool slots = d == 0 && K;  // the ingress identity includes the pod's job descriptors
    std::fill(slot_pod.begin(), slot_pod.end(), UINT32_MAX);
    for (uint32_t p = 0; p < pb.P; p++) {
      uint64_t h = hmix((uint64_t(pb.pod_ns[p]) << 32) | pb.pod_ls[p]);
      if (slots)
        for (uint32_t k = 0; k < K; k++)
          h = hmix(h ^ (uint64_t(uint32_t(pb.slot_desc[size_t(p) * K + k])) << 8 | pb.slot_status[size_t(p) * K + k]));
      uint32_t x = uint32_t(h) & (cap - 1);
      for (;; x = (x + 1) & (cap - 1)) {
        const uint32_t q = slot_pod[x];
        if (q == UINT32_MAX) break;
        if (pb.pod_ns[q] == pb.pod_ns[p] && pb.pod_ls[q] == pb.pod_ls[p] &&
            (!slots || (memcmp(&pb.slot_desc[size_t(q) * K], &pb.slot_desc[size_t(p) * K], 4 * size_t(K)) == 0 &&
                        memcmp(&pb.slot_status[size_t(q) * K], &pb.slot_status[size_t(p) * K], K) == 0)))
          break;
      }
      if (slot_pod[x] == UINT32_MAX) {
        slot_pod[x] = p;
        slot_id[x] = uint32_t(I.ns.size());
        I.ns.push_back(pb.pod_ns[p]);
        I.ls.push_back(pb.pod_ls[p]);
        I.nsls.push_back(pb.pod_nsls[p]);
        if (d == 0)
          for (uint32_t k = 0; k < K; k++) {
            I.desc.push_back(pb.slot_desc[size_t(p) * K + k]);
            I.status.push_back(pb.slot_status[size_t(p) * K + k]);
          }
      }
      I.of_pod[p] = slot_id[x];
    }
    I.list_off.resize(I.ns.size());
    uint64_t tot = 0;
    for (size_t i = 0; i < I.ns.size(); i++) {
      I.list_off[i] = uint32_t(tot);
      tot += pb.tns_hi[d][I.ns[i]] - pb.tns_lo[d][I.ns[i]];
      if (tot > 0xFFFFFFFFull) throw Panic{CYC_ERR_OOM, "membership lists exceed 2^32 entries"};
    }
    I.list_total = tot;
    uint32_t hc = 2;
    while (hc < 2 * I.ns.size()) hc <<= 1;
    I.ht_cap = hc;
  }
}

// Host side of the peer-row stage: which peers are pod peers / IP peers, and for every 64-pod
// word the runs of equal egress identity (a pod peer's outcome is a function of that identity).
static PeerPlan plan_peers(const Problem& pb, const Identities& eg) {
  PeerPlan pl;
  for (uint32_t j = 0; j < pb.peers.size(); j++) {
    if (pb.peers[j].kind == PK_POD) pl.pod_peers.push_back(j);
    else if (pb.peers[j].kind == PK_IP) {
      pl.ip_peers.push_back(j);
      const DIPBlock& b = pb.ipbs[pb.peers[j].ipb];
      DIPTest t{};
      t.peer = j;
      t.exoff = uint32_t(pl.ip_ex.size());
      t.excnt = b.excnt;
      t.cidr = pb.cidrs[b.cidr];
      for (uint32_t e = 0; e < b.excnt; e++) pl.ip_ex.push_back(pb.cidrs[pb.ipb_ex[b.exoff + e]]);
      pl.ip_tests.push_back(t);
    }
  }
  pl.word_off.push_back(0);
  for (uint32_t w = 0; w < pb.W; w++) {
    uint32_t q0 = w * 64, q1 = std::min<uint32_t>(pb.P, q0 + 64);
    for (uint32_t q = q0; q < q1; q++) {
      uint32_t e = eg.of_pod[q];
      size_t start = pl.word_off.back();
      size_t x = pl.run_e.size();
      // merge with an earlier run of the same identity in this word (keeps runs short)
      size_t hit = x;
      for (size_t y = start; y < x; y++)
        if (pl.run_e[y] == e) {
          hit = y;
          break;
        }
      if (hit == x) {
        pl.run_e.push_back(e);
        pl.run_mask.push_back(0);
      }
      pl.run_mask[hit] |= 1ull << (q - q0);
    }
    pl.word_off.push_back(uint32_t(pl.run_e.size()));
    pl.max_runs = std::max(pl.max_runs, pl.word_off.back() - pl.word_off[pl.word_off.size() - 2]);
  }
  if (pl.max_runs <= IDO_MAX_RUNS) {
    pl.runs.assign(pb.W, WordRuns{});
    for (uint32_t w = 0; w < pb.W; w++)
      for (uint32_t x = pl.word_off[w]; x < pl.word_off[w + 1]; x++) {
        pl.runs[w].e[x - pl.word_off[w]] = pl.run_e[x];
        pl.runs[w].m[x - pl.word_off[w]] = pl.run_mask[x];
      }
  }
  return pl;
}

static uint64_t ido_b_bytes(const cyc_ctx* c, int d) {
  const uint64_t EW = (c->ids[1].ns.size() + 63) / 64, D = std::max<size_t>(c->pb.descs.size(), 1);
  return uint64_t(c->ids[d].ns.size()) * (d == 0 ? c->pb.K : D) * EW * 8;
}

static uint64_t ido_lds_bytes(const cyc_ctx* c) {  // k_class_rows_ido: staged identity-set rows
  const uint64_t EW = (c->ids[1].ns.size() + 63) / 64, D = std::max<size_t>(c->pb.descs.size(), 1);
  return std::max<uint64_t>(std::min<uint64_t>(8, c->pb.K), D) * EW * 8;  // KC <= 8 slot rows or D
}

static bool ido_possible(const cyc_ctx* c) {
  return !c->pb.may_err && c->plan.max_runs <= IDO_MAX_RUNS && ido_lds_bytes(c) <= IDO_LDS_BYTES &&
         ido_b_bytes(c, 0) + ido_b_bytes(c, 1) <= (1ull << 30);
}

// Batched blocks: per block (first pod, pods, first slot, slots) and its output slab offsets; per
// identity its block and class-row window (its block's words).
static void prepare_blocks_device(cyc_ctx* c) {
  Problem& pb = c->pb;
  c->blk_off_h.clear();
  c->blk_wa_max = c->blk_np_max = 0;
  if (pb.blocks.empty()) return;
  std::vector<uint32_t> cfg_k0(pb.n_cfg + 1, pb.K), cfg_nk(pb.n_cfg, 0);
  for (uint32_t k = pb.K; k-- > 0;) cfg_k0[pb.slot_cfg[k]] = k;
  for (uint32_t k = 0; k < pb.K; k++) cfg_nk[pb.slot_cfg[k]]++;
  std::vector<uint4> bl(pb.blocks.size());
  uint64_t words = 0, bytes = 0;
  for (size_t b = 0; b < pb.blocks.size(); b++) {
    const ProbeBlock& x = pb.blocks[b];
    const uint32_t np = x.p1 - x.p0, nk = cfg_nk[x.cfg];
    bl[b] = uint4{x.p0, np, cfg_k0[x.cfg], nk};
    c->blk_off_h.push_back(words);
    c->blk_off_h.push_back(bytes);
    words += uint64_t(np) * nk * ((np + 63) / 64);
    bytes += uint64_t(np) * nk;
    c->blk_wa_max = std::max<uint32_t>(c->blk_wa_max, np ? (x.p1 + 63) / 64 - x.p0 / 64 : 0u);
    c->blk_np_max = std::max(c->blk_np_max, np);
  }
  c->blk_off_h.push_back(words);
  c->blk_off_h.push_back(bytes);
  upload(c->blk, bl);
  upload(c->blk_off, c->blk_off_h);
  for (int d = 0; d < 2; d++) {
    const Identities& I = c->ids[d];
    std::vector<uint32_t> ib(I.ns.size(), 0);
    std::vector<uint2> iw(I.ns.size(), uint2{0, 0});
    for (uint32_t q = 0; q < pb.P; q++) {
      const ProbeBlock& x = pb.blocks[pb.pod_blk[q]];
      ib[I.of_pod[q]] = pb.pod_blk[q];
      iw[I.of_pod[q]] = uint2{x.p0 / 64, (x.p1 + 63) / 64 - x.p0 / 64};
    }
    upload(c->id_blk[d], ib);
    upload(c->id_win[d], iw);
  }
  c->first_blk.alloc(std::max<uint64_t>(pb.blocks.size() * 8, 16));
}

static void prepare_device(cyc_ctx* c) {
  Problem& pb = c->pb;
  PhaseClock clk("prepare_device");
  upload(c->ls_off, pb.ls_off);
  upload(c->ls_key, pb.ls_key);
  upload(c->ls_val, pb.ls_val);
  upload(c->sel_off, pb.sel_off);
  upload(c->reqs, pb.reqs);
  upload(c->req_vals, pb.req_vals);
  upload(c->pod_ns, pb.pod_ns);
  upload(c->pod_ls, pb.pod_ls);
  upload(c->pod_nsls, pb.pod_nsls);
  upload(c->pod_ip, pb.pod_ip);
  {  // the address index of the range-built IP rows: IPv4 pods by address, then IPv6 pods
    std::vector<uint32_t> p4, p6;
    for (uint32_t q = 0; q < pb.P; q++)
      if (pb.pod_ip[q].valid) (pb.pod_ip[q].fam == 4 ? p4 : p6).push_back(q);
    std::stable_sort(p4.begin(), p4.end(), [&](uint32_t x, uint32_t y) { return pb.pod_ip[x].w[3] < pb.pod_ip[y].w[3]; });
    auto a6 = [&](uint32_t q) { return std::array<uint32_t, 4>{pb.pod_ip[q].w[0], pb.pod_ip[q].w[1], pb.pod_ip[q].w[2], pb.pod_ip[q].w[3]}; };
    std::stable_sort(p6.begin(), p6.end(), [&](uint32_t x, uint32_t y) { return a6(x) < a6(y); });
    c->ip4_key.resize(p4.size());
    c->ip6_key.resize(p6.size());
    for (size_t x = 0; x < p4.size(); x++) c->ip4_key[x] = pb.pod_ip[p4[x]].w[3];
    for (size_t x = 0; x < p6.size(); x++) c->ip6_key[x] = a6(p6[x]);
    c->ipsort_host = p4;
    c->ipsort_host.insert(c->ipsort_host.end(), p6.begin(), p6.end());
    upload(c->ipsort, c->ipsort_host);
    // a family whose pods' addresses never decrease in pod order (addresses handed out in pod order:
    // configs #2-#4) sorts to pod order, so its sorted positions ARE its pods in pod order: a network's
    // pods of that family are then pod-index intervals (ip_rows_iv_blk)
    auto mono = [](const std::vector<uint32_t>& pods) {
      for (size_t x = 1; x < pods.size(); x++)
        if (pods[x] < pods[x - 1]) return false;
      return true;
    };
    c->ip_mono[0] = mono(p4);
    c->ip_mono[1] = mono(p6);
  }
  upload(c->cidrs, pb.cidrs);
  upload(c->ipbs, pb.ipbs);
  upload(c->ipb_ex, pb.ipb_ex);
  upload(c->pms, pb.pms);
  upload(c->pents, pb.pents);
  upload(c->peers, pb.peers);
  upload(c->descs, pb.descs);
  upload(c->slot_desc, pb.slot_desc);
  upload(c->slot_status, pb.slot_status);
  upload(c->slot_cfg, pb.slot_cfg);
  upload(c->slot_idx, pb.slot_idx);
  clk.lap("uploads");
  uint64_t R = pb.peers.size(), W = pb.W, D = std::max<size_t>(pb.descs.size(), 1), K = pb.K;
  c->selres.alloc(std::max<uint64_t>(uint64_t(pb.S) * pb.L, 16));
  {  // dense label table for k_selectors_dense: label keys -> dense index kx, LVT[kx][l]
    std::vector<int32_t> kx(pb.strings.size(), -1);
    uint32_t nk = 0;
    for (uint32_t k : pb.ls_key)
      if (kx[k] < 0) kx[k] = int32_t(nk++);
    c->dense_sel = uint64_t(nk + 1) * pb.L * 4 <= (256ull << 20);
    c->sel_one_h.clear();
    if (c->dense_sel) {
      std::vector<uint32_t> lvt(uint64_t(nk + 1) * pb.L, 0xFFFFFFFFu);
      for (uint32_t l = 0; l < pb.L; l++)
        for (uint32_t x = pb.ls_off[l]; x < pb.ls_off[l + 1]; x++) lvt[uint64_t(kx[pb.ls_key[x]]) * pb.L + l] = pb.ls_val[x];
      std::vector<DReq> dr = pb.reqs;
      for (DReq& q : dr) q.key = (q.op != REQ_INVALID && q.key < kx.size() && kx[q.key] >= 0) ? uint32_t(kx[q.key]) : nk;
      upload(c->lvt, lvt);
      upload(c->dreqs, dr);
      {  // one-requirement selectors in a single record each (SelView::one)
        std::vector<uint4> one(std::max<size_t>(pb.S, 1), uint4{SEL_WALK, 0, 0, 0});
        for (uint32_t sid = 0; sid < pb.S; sid++) {
          const uint32_t r0 = pb.sel_off[sid], nr = pb.sel_off[sid + 1] - r0;
          if (nr == 0) {
            one[sid].x = SEL_ALL;
            continue;
          }
          const DReq& q = dr[r0];
          if (nr != 1 || q.op == REQ_INVALID || q.vcnt > 2) continue;
          const bool has_v = q.op == REQ_EQ || q.op == REQ_EQ_EMPTY || q.op == REQ_IN || q.op == REQ_NOTIN;
          const uint32_t vc = has_v ? (q.op == REQ_EQ || q.op == REQ_EQ_EMPTY ? 1u : q.vcnt) : 0u;
          one[sid] = uint4{q.op | (vc << 8), q.key, vc > 0 ? pb.req_vals[q.voff] : 0u, vc > 1 ? pb.req_vals[q.voff + 1] : 0u};
        }
        upload(c->sel_one, one);
        c->sel_one_h = one;
      }
      // the same table per pod (PLVT, sparse pod-peer rows) is gathered on the device when a run
      // first needs it (ensure_plvt): IDO builds never read it, and it is (keys + 1) x P words
      c->n_lkeys = nk;
      c->plvt.alloc(0);
      c->plvt_ready = false;
      // label postings: the pods under each (dense key, value) of their own labels, and per EQ / IN
      // (<= 2 values) requirement the postings of its values (pod_rows_post_blk)
      // (key, value, pod) triples sorted by (key, value), pods ascending within: two counting-sort
      // passes (value, then key; both are dictionary ids), O(pairs + dictionary)
      std::vector<std::pair<uint64_t, uint32_t>> kv;
      {
        const size_t NV = pb.strings.size() + 1, NK = nk + 1;
        size_t n = 0;
        for (uint32_t q = 0; q < pb.P; q++) n += pb.ls_off[pb.pod_ls[q] + 1] - pb.ls_off[pb.pod_ls[q]];
        std::vector<uint32_t> kk(n), vv(n), qq(n), cnt(std::max(NV, NK) + 1);
        size_t x0 = 0;
        for (uint32_t q = 0; q < pb.P; q++) {
          const uint32_t l = pb.pod_ls[q];
          for (uint32_t x = pb.ls_off[l]; x < pb.ls_off[l + 1]; x++, x0++) {
            kk[x0] = uint32_t(kx[pb.ls_key[x]]);
            vv[x0] = pb.ls_val[x];
            qq[x0] = q;
          }
        }
        std::vector<uint32_t> ord(n), ord2(n);
        auto pass = [&](const std::vector<uint32_t>& key, size_t range, const std::vector<uint32_t>& in, std::vector<uint32_t>& out) {
          std::fill(cnt.begin(), cnt.begin() + range + 1, 0u);
          for (uint32_t i : in) cnt[key[i] + 1]++;
          for (size_t r = 0; r < range; r++) cnt[r + 1] += cnt[r];
          for (uint32_t i : in) out[cnt[key[i]]++] = i;
        };
        std::iota(ord.begin(), ord.end(), 0u);  // pod order (q ascending)
        pass(vv, NV, ord, ord2);
        pass(kk, NK, ord2, ord);
        kv.resize(n);
        for (size_t i = 0; i < n; i++) kv[i] = {(uint64_t(kk[ord[i]]) << 32) | vv[ord[i]], qq[ord[i]]};
      }
      std::vector<uint32_t> pods(kv.size());
      for (size_t i = 0; i < kv.size(); i++) pods[i] = kv[i].second;
      auto range = [&](uint32_t key, uint32_t v) {
        const uint64_t k = (uint64_t(key) << 32) | v;
        auto lo = std::lower_bound(kv.begin(), kv.end(), std::make_pair(k, 0u));
        auto hi = std::lower_bound(kv.begin(), kv.end(), std::make_pair(k + 1, 0u));
        return std::make_pair(uint32_t(lo - kv.begin()), uint32_t(hi - lo));
      };
      std::vector<uint4> rp(dr.size(), uint4{0, 0, 0, 0});
      c->req_post_ok.assign(dr.size(), 0);
      for (size_t r = 0; r < dr.size(); r++) {
        const DReq& q = dr[r];
        if (q.key >= nk || !(q.op == REQ_EQ || (q.op == REQ_IN && q.vcnt >= 1 && q.vcnt <= 2))) continue;
        const auto a = range(q.key, pb.req_vals[q.voff]);
        rp[r] = uint4{a.first, a.second, 0, 0};
        if (q.op == REQ_IN && q.vcnt == 2 && pb.req_vals[q.voff + 1] != pb.req_vals[q.voff]) {
          const auto b = range(q.key, pb.req_vals[q.voff + 1]);
          rp[r].z = b.first;
          rp[r].w = b.second;
        }
        c->req_post_ok[r] = 1;
      }
      upload(c->req_post, rp);
      upload(c->post_pods, pods);
    }
  }
  clk.lap("label tables");
  c->PM.alloc(std::max<uint64_t>(R * W * 8, 16));
  c->ip_rng.alloc(std::max<uint64_t>(R * 16 + R * ((W + 63) / 64) * 4, 16));  // [R][4] word spans + chunk masks, then [R][W/64] cnz
  c->ip_rng_clean = false;  // a new buffer: the next fused front fills it (no emit has reset it yet)
  c->ER.alloc(pb.may_err ? std::max<uint64_t>(R * W * 8, 16) : 16);
  {
    c->plan = plan_peers(pb, c->ids[1]);
    PeerPlan& pl = c->plan;
    upload(c->word_off, pl.word_off);
    upload(c->run_e, pl.run_e);
    upload(c->run_mask, pl.run_mask);
    upload(c->runs, pl.runs);
    upload(c->id_nsls, c->ids[1].nsls);
    {  // per-word, per-family address intervals for k_ip_rows_fast, then one record per 64-word chunk
      const uint32_t NC = (pb.W + 63) / 64;
      std::vector<DWordIP> wi(pb.W + NC);
      c->word_aff.assign(pb.W, 3);
      for (uint32_t w = 0; w < pb.W; w++) {
        DWordIP d{};
        d.min4 = 0xFFFFFFFFu;
        for (int i = 0; i < 4; i++) d.min6[i] = 0xFFFFFFFFu;
        // affine check per family: every pod of the family at lane i holds base + i (128-bit, big-endian
        // words; v4 in w[3]) for one base (DWordIP::aff)
        bool aff[2] = {true, true};
        int first[2] = {-1, -1};
        uint32_t base[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
        for (uint32_t q = w * 64; q < std::min<uint32_t>(pb.P, w * 64 + 64); q++) {
          const DIP& ip = pb.pod_ip[q];
          if (!ip.valid) continue;  // only with may_err, where the fast kernel is not used
          const uint32_t lane = q - w * 64;
          const int f = ip.fam == 4 ? 0 : 1;
          uint32_t a[4] = {f ? ip.w[0] : 0u, f ? ip.w[1] : 0u, f ? ip.w[2] : 0u, ip.w[3]};
          // b = a - lane (128-bit): the pod's base
          uint32_t b[4];
          uint64_t borrow = lane;
          for (int i = 3; i >= 0; i--) {
            const uint64_t v = uint64_t(a[i]) - borrow;
            b[i] = uint32_t(v);
            borrow = (v >> 63) & 1u;  // went below zero
          }
          if (borrow) aff[f] = false;  // address < lane: no base (never affine)
          if (first[f] < 0) {
            first[f] = int(lane);
            std::copy(b, b + 4, base[f]);
          } else if (!std::equal(b, b + 4, base[f])) {
            aff[f] = false;
          }
          if (ip.fam == 4) {
            d.m4 |= 1ull << lane;
            d.min4 = std::min(d.min4, ip.w[3]);
            d.max4 = std::max(d.max4, ip.w[3]);
          } else {
            d.m6 |= 1ull << lane;
            if (std::lexicographical_compare(ip.w, ip.w + 4, d.min6, d.min6 + 4)) std::copy(ip.w, ip.w + 4, d.min6);
            if (std::lexicographical_compare(d.max6, d.max6 + 4, ip.w, ip.w + 4)) std::copy(ip.w, ip.w + 4, d.max6);
          }
        }
        for (int f = 0; f < 2; f++)
          if (first[f] >= 0 && aff[f]) d.aff |= (uint32_t(first[f]) | 0x80u) << (8 * f);
        c->word_aff[w] = uint8_t((first[0] < 0 || aff[0] ? 1u : 0u) | (first[1] < 0 || aff[1] ? 2u : 0u));
        wi[w] = d;
      }
      for (uint32_t ch = 0; ch < NC; ch++) {
        DWordIP d{};
        d.min4 = 0xFFFFFFFFu;
        for (int i = 0; i < 4; i++) d.min6[i] = 0xFFFFFFFFu;
        for (uint32_t w = ch * 64; w < std::min<uint32_t>(pb.W, ch * 64 + 64); w++) {
          const DWordIP& x = wi[w];
          if (x.m4) {
            d.m4 |= 1ull << (w - ch * 64);
            d.min4 = std::min(d.min4, x.min4);
            d.max4 = std::max(d.max4, x.max4);
          }
          if (x.m6) {
            d.m6 |= 1ull << (w - ch * 64);
            if (std::lexicographical_compare(x.min6, x.min6 + 4, d.min6, d.min6 + 4)) std::copy(x.min6, x.min6 + 4, d.min6);
            if (std::lexicographical_compare(d.max6, d.max6 + 4, x.max6, x.max6 + 4)) std::copy(x.max6, x.max6 + 4, d.max6);
          }
        }
        wi[pb.W + ch] = d;
      }
      upload(c->ip_words, wi);
      c->ipw_h = wi;
      // namespace range of every word's and chunk's pods (pod_rows_sparse_blk)
      std::vector<DWordNS> nw(pb.W + NC, DWordNS{0xFFFFFFFFu, 0u, 0u, 0u});
      for (uint32_t q = 0; q < pb.P; q++) {
        for (DWordNS* x : {&nw[q / 64], &nw[pb.W + q / 4096]}) {
          if (x->lo == 0xFFFFFFFFu) x->nsls = pb.pod_nsls[q];
          else if (x->lo != pb.pod_ns[q] || x->hi != pb.pod_ns[q]) x->nsls = 0xFFFFFFFFu;
          x->lo = std::min(x->lo, pb.pod_ns[q]);
          x->hi = std::max(x->hi, pb.pod_ns[q]);
        }
      }
      upload(c->ns_words, nw);
    }
    c->ido.alloc(std::max<uint64_t>(uint64_t(pl.pod_peers.size()) * c->ids[1].ns.size(), 16));
    c->idob.alloc(std::max<uint64_t>(uint64_t(pl.pod_peers.size()) * ((c->ids[1].ns.size() + 63) / 64) * 8, 16));
  }
  clk.lap("peer plan");
  {  // one VALID descriptor per slot across all pods? (egress class rows then skip the per-word slot words)
    std::vector<int32_t> ud(std::max<uint32_t>(pb.K, 1), -1);
    bool uni = pb.P > 0 && pb.K > 0;
    for (uint32_t k = 0; k < pb.K && uni; k++) {
      ud[k] = pb.slot_desc[k];
      for (uint32_t q = 0; q < pb.P && uni; q++)
        uni = pb.slot_status[size_t(q) * pb.K + k] == CYC_JOB_VALID && pb.slot_desc[size_t(q) * pb.K + k] == ud[k];
    }
    c->uni_desc = uni;
    upload(c->udesc, ud);
  }
  c->portok.alloc(std::max<uint64_t>(pb.pms.size() * D, 16));
  c->portbits.alloc(std::max<uint64_t>(pb.pms.size() * 4, 16));
  c->VALID.alloc(std::max<uint64_t>(K * W * 8, 16));
  c->DESCW.alloc(std::max<uint64_t>(K * W * 4, 16));
  c->DM.alloc(std::max<uint64_t>(K * D * W * 8, 16));
  c->first_err.alloc(std::max<uint64_t>(uint64_t(pb.n_cfg) * 8, 16));  // per probe config (k_first_error)
  c->status_sink.alloc(std::max<uint64_t>(uint64_t(pb.P) * K, 16));
  for (int d = 0; d < 2; d++) {
    Identities& I = c->ids[d];
    DirDev& dd = c->dir[d];
    dd.n = uint32_t(I.ns.size());
    dd.ht_cap = I.ht_cap;
    upload(dd.id_ns, I.ns);
    upload(dd.id_ls, I.ls);
    upload(dd.id_desc, I.desc);
    upload(dd.id_status, I.status);
    upload(dd.list_off, I.list_off);
    upload(dd.tns_lo, pb.tns_lo[d]);
    upload(dd.tns_hi, pb.tns_hi[d]);
    upload(dd.tgt, pb.tgt[d]);
    upload(dd.pod_id, I.of_pod);
    dd.list.alloc(std::max<uint64_t>(I.list_total * 4, 16));
    dd.cnt.alloc(std::max<uint64_t>(dd.n * 4ull, 16));
    dd.hash.alloc(std::max<uint64_t>(dd.n * 8ull, 16));
    dd.err.alloc(std::max<uint64_t>(dd.n, 16));
    dd.ht_key.alloc(uint64_t(dd.ht_cap) * 16 + 16);  // [cap] 16-byte entries (key ~0 = empty, rep), counter
    HIPCHK(hipMemset(dd.ht_key.p, 0xFF, dd.ht_key.bytes));  // empty; afterwards every run's class rows empty it
    if (!c->zeros.p) {
      c->zeros.alloc(256);
      HIPCHK(hipMemset(c->zeros.p, 0, 256));
    }
    dd.reps.alloc(std::max<uint64_t>(dd.n * 4ull, 16));
    dd.class_of.alloc(std::max<uint64_t>(dd.n * 4ull, 16));
    dd.A.alloc(std::max<uint64_t>(uint64_t(dd.n) * K * W * 8, 16));
    if (pb.may_err) dd.AE.alloc(std::max<uint64_t>(uint64_t(dd.n) * K * W * 8, 16));
    else dd.AE.alloc(0);
    dd.B.alloc(ido_possible(c) ? std::max<uint64_t>(ido_b_bytes(c, d), 16) : 16);
    {  // IP-peer list bounds per identity: the IP peers of its namespace's targets
      // (upper bound for both list uses: IDO builds list the IP peers, PM builds every peer)
      std::vector<uint32_t> ns_ip(pb.strings.size(), 0), off(dd.n + 1, 0);
      for (const DTarget& t : pb.tgt[d]) ns_ip[t.ns] += t.pcnt;
      for (uint32_t i = 0; i < dd.n; i++) off[i + 1] = off[i] + ns_ip[I.ns[i]];
      upload(dd.ip_off, off);
      dd.ip_cnt.alloc(std::max<uint64_t>(dd.n * 4ull, 16));
      dd.ip_list.alloc(std::max<uint64_t>(uint64_t(off[dd.n]) * 16, 16));
    }
  }
  clk.lap("scratch");
  prepare_blocks_device(c);
  c->order_lo = c->order_hi = -1;
  c->order_src = false;
}

// nonzero-chunk flags of the IP peers' PM rows, after the word spans and chunk masks in the ip_rng buffer
static uint32_t* ip_cnz(cyc_ctx* c) { return c->ip_rng.as<uint32_t>() + 4 * c->pb.peers.size(); }

static unsigned grid1(uint64_t n, unsigned block) { return unsigned(std::min<uint64_t>((n + block - 1) / block, 1u << 20)); }

static bool front_fused_ok(const cyc_ctx* c);
static bool ido_mode(const cyc_ctx* c);
// Selectors evaluated where used (sel_at through LVT), not as the dense SELRES table: the fused
// front of PM builds (its pod-peer rows and membership are the only selector users, and PM builds
// are the ones whose label sets number ~ the pods).  The DAG path computes SELRES regardless.
// PM builds' fused front: sparse pod-peer rows (pod_rows_sparse_blk, launch C) once the rows are
// large (>= 2M pod-peer words: config #3u), else full rows a wave per (pod peer, word) in launch B,
// which has the parallelism small problems need (config #2: 125k peer words, B + C 33 vs 52 us).
// pr_group > 0 forces the sparse rows.
static bool pod_sparse(const cyc_ctx* c) {
  if (ido_mode(c)) return false;
  const uint64_t Rp = c->rp_off[2] - c->rp_off[0];
  return c->pr_group > 0 || Rp * c->pb.W >= (2ull << 20);
}
// PLVT (each pod's value of every dense label key) for the sparse pod-peer rows: gathered on the
// device from LVT once per prepare, on the run's stream ahead of the step, when a run needs it
// and it fits PLVT_MAX_BYTES; otherwise the rows read LVT through each pod's label set (SelView
// with PLVT null), one more dependent load per pod.
static void ensure_plvt(cyc_ctx* c, hipStream_t st) {
  if (c->plvt_ready || !c->dense_sel || !pod_sparse(c)) return;
  const uint64_t n = uint64_t(c->n_lkeys + 1) * c->pb.P;
  if (!n || n * 4 > (uint64_t(c->plvt_max_mb) << 20)) return;
  c->plvt.alloc(n * 4);
  k_plvt<<<grid1(n, 256), 256, 0, st>>>(c->lvt.as<uint32_t>(), c->pod_ls.as<uint32_t>(), c->pb.L, c->pb.P, n,
                                        c->plvt.as<uint32_t>());
  HIPCHK(hipGetLastError());
  c->plvt_ready = true;
}
static bool lazy_sel(const cyc_ctx* c) {
  if (!c->dense_sel || c->pb.may_err || c->sel_lazy == 0 || !front_fused_ok(c)) return false;
  const bool pod_peers = c->rp_off[2] > c->rp_off[0];
  // no pod-peer rows at all (IPBlock-only policies, config #4): the membership is the only selector
  // user, one record and one label-table load per target — no table, and no launch A
  if (!pod_peers && c->sel_lazy < 0) return true;
  // auto: lazy once the dense table would take ~0.1 ms (>= 64M pairs; config #3u: 0.75G pairs,
  // 1.1 ms; config #2 stays dense — its multi-requirement selectors cost more evaluated per use)
  // IDO builds always: their identity sets and membership evaluate fewer pairs than the table
  // holds (config #3: A + B 118 -> 111 us; its N = 8 shard 35 -> 31 us, profiles/r02_sel_lazy_ab.txt)
  return c->sel_lazy == 1 || ido_mode(c) || uint64_t(c->n_sel) * c->pb.L >= (64ull << 20);
}
static SelView sel_view(cyc_ctx* c) {
  SelView v{};
  v.selres = lazy_sel(c) ? nullptr : c->selres.as<uint8_t>();
  v.L = c->pb.L;
  v.sel_off = c->sel_off.as<uint32_t>();
  v.req_vals = c->req_vals.as<uint32_t>();
  v.LVT = c->lvt.as<uint32_t>();
  v.dreqs = c->dreqs.as<DReq>();
  v.PLVT = c->plvt_ready ? c->plvt.as<uint32_t>() : nullptr;  // null: pod -> label set -> LVT gathers
  v.P = c->pb.P;
  v.one = c->sel_one.as<uint4>();
  return v;
}

static MemberArgs member_args(cyc_ctx* c, int d) {
  Problem& pb = c->pb;
  DirDev& dd = c->dir[d];
  MemberArgs a{};
  a.n_ident = dd.n;
  a.L = pb.L;
  a.K = pb.K;
  a.id_ns = dd.id_ns.as<uint32_t>();
  a.id_ls = dd.id_ls.as<uint32_t>();
  a.id_desc = d == 0 ? dd.id_desc.as<int32_t>() : nullptr;
  a.id_status = d == 0 ? dd.id_status.as<uint8_t>() : nullptr;
  a.tns_lo = dd.tns_lo.as<uint32_t>();
  a.tns_hi = dd.tns_hi.as<uint32_t>();
  a.tgt = dd.tgt.as<DTarget>();
  a.sv = sel_view(c);
  a.list_off = dd.list_off.as<uint32_t>();
  a.list = dd.list.as<uint32_t>();
  a.cnt = dd.cnt.as<uint32_t>();
  a.hash = dd.hash.as<uint64_t>();
  a.err = dd.err.as<uint8_t>();
  a.ht_key = dd.ht_key.as<unsigned long long>();
  a.ht_cap = dd.ht_cap;
  a.act = c->act[d].as<uint32_t>();
  a.actrec = c->actrec[d].as<uint4>();
  a.n_act = c->n_act[d];
  a.reps = dd.reps.as<uint32_t>();
  a.rep_cnt = dd.rep_cnt();
  a.id_blk = c->pb.blocks.empty() ? nullptr : c->id_blk[d].as<uint32_t>();
  return a;
}

// PM-build class rows (k_class_rows_pl): threads per block — PL_THREADS, or 256 for rows of >= 16
// chunks (the wave-per-chunk rows then split a class's chunks over 4 waves: config #3u -5 %,
// config #4's 13 chunks +9 %: profiles/r02_pl_threads_ab.txt) — and blocks per direction, striding
// over the representatives, about two blocks in flight per CU slot
static uint32_t pl_threads(const cyc_ctx* c) { return (c->pb.W + 63) / 64 >= 16 ? 256u : PL_THREADS; }
static uint32_t pl_blocks(const cyc_ctx* c, int d) { return std::min<uint32_t>(c->n_act[d], 2048u * 256u / pl_threads(c)); }

// Range plan for rows [lo,hi): (1) the rows ordered so pods sharing class rows are adjacent
// (L2 / Infinity-Cache reuse in k_emit); (2) the identities those rows use, per direction —
// only their classes are elected and their class rows computed; (3) the peers of the targets
// in those identities' namespaces — only their PM rows are built.  A rank of an N-GPU run thus
// does ~1/N of the front work too, not just 1/N of the emit.
// Source-row plans (src): rows [lo, hi) are SOURCES; the run computes every cell (s in [lo, hi), d,
// k): egress rows of sources [lo, hi) (full rows) and the ingress rows of EVERY destination, but
// only their words [lo / 64, ceil(hi / 64)) — the shard's sources as peers.  lo must be a multiple
// of 64 and hi too unless it is P (checked by the caller), so the windows of a partition tile the words.
static void peer_chunks(const cyc_ctx* c, int d, uint32_t& c0, uint32_t& nch);
static bool one_window(const cyc_ctx* c);
// Host restatement of ip_rows_fast_blk's chunk test: false when network n misses the chunk's pods'
// addresses of its family (or the chunk has none of that family).
static bool ip_chunk_touch(const DCidr& n, const DWordIP& ck) {
  if (!n.valid) return true;
  if (n.fam == 4) {
    const uint32_t lo = n.net[3] & n.mask[3], hi = lo | ~n.mask[3];
    return ck.m4 && !(ck.max4 < lo || ck.min4 > hi);
  }
  uint32_t lo[4], hi[4];
  for (int i = 0; i < 4; i++) {
    lo[i] = n.net[i] & n.mask[i];
    hi[i] = lo[i] | ~n.mask[i];
  }
  auto lt = [](const uint32_t* a, const uint32_t* b) { return std::lexicographical_compare(a, a + 4, b, b + 4); };
  return ck.m6 && !(lt(ck.max6, lo) || lt(hi, ck.min6));
}

static void ensure_range(cyc_ctx* c, int64_t lo, int64_t hi, bool src = false) {
  if (c->order_lo == lo && c->order_hi == hi && c->order_src == src) return;
  Problem& pb = c->pb;
  PhaseClock clk("range plan");
  c->rl[0] = src ? 0 : lo;
  c->rh[0] = src ? int64_t(pb.P) : hi;
  c->rl[1] = lo;
  c->rh[1] = hi;
  c->win_w0 = src ? uint32_t(lo / 64) : 0u;
  c->win_wa = src ? uint32_t((hi + 63) / 64 - lo / 64) : pb.W;
  if (src && hi <= lo) c->win_wa = 0;
  {  // the egress identities of the window's pods (identity ids follow first appearance in pod order, so a
     // source shard's are mostly one range): the ingress identity sets need only their words
    const uint32_t EW = uint32_t((c->ids[1].ns.size() + 63) / 64);
    c->ido_ew0 = 0;
    c->ido_ew1 = EW;
    if (src) {
      uint32_t e0 = UINT32_MAX, e1 = 0;
      for (int64_t q = c->win_w0 * 64ll; q < std::min<int64_t>(int64_t(c->win_w0 + c->win_wa) * 64, pb.P); q++) {
        e0 = std::min(e0, c->ids[1].of_pod[size_t(q)]);
        e1 = std::max(e1, c->ids[1].of_pod[size_t(q)] + 1);
      }
      c->ido_ew0 = e0 == UINT32_MAX ? 0u : e0 / 64;
      c->ido_ew1 = e0 == UINT32_MAX ? 0u : (e1 + 63) / 64;
    }
  }
  // row phases (cyc_ctx::row_phases): a whole no-panic table splits at row P/2 — auto once each plane
  // is >= 8 GB; the emit lists then hold the rows before the split first
  const bool whole = lo == 0 && hi == int64_t(pb.P) && (!src || c->win_wa == pb.W);
  const bool big = uint64_t(pb.P) * pb.K * pb.W * 8 >= (8ull << 30);
  c->phase_split = c->row_phases != 1 && whole && !pb.may_err && pb.blocks.empty() && pb.P >= 128 &&
                           (c->row_phases == 2 || big) ? uint32_t(pb.P / 2) : 0u;
  for (int d = 0; d < 2; d++) {  // emit row order: clustered by this direction's identity, (pod, identity) pairs
    std::vector<uint32_t> ord(size_t(c->rh[d] - c->rl[d]));
    std::iota(ord.begin(), ord.end(), uint32_t(c->rl[d]));
    const auto& i1 = c->ids[d].of_pod;
    const auto& i2 = c->ids[1 - d].of_pod;
    const uint32_t split = c->phase_split;
    std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) {
      if (split && (x < split) != (y < split)) return x < split;
      return i1[x] != i1[y] ? i1[x] < i1[y] : i2[x] < i2[y];
    });
    c->phase_n1[d] = split ? split - uint32_t(c->rl[d]) : 0u;
    std::vector<uint32_t> pairs(ord.size() * 2);
    for (size_t r = 0; r < ord.size(); r++) {
      pairs[2 * r] = ord[r];
      pairs[2 * r + 1] = i1[ord[r]];
    }
    upload(c->order[d], pairs);
  }
  std::vector<uint8_t> peer_needed(pb.peers.size(), 0), peer_dir(pb.peers.size(), 0);
  for (const DTarget& t : pb.tgt[1])
    for (uint32_t j = t.poff; j < t.poff + t.pcnt; j++) peer_dir[j] = 1;
  for (int d = 0; d < 2; d++) {
    const Identities& I = c->ids[d];
    std::vector<uint8_t> used(I.ns.size(), 0);
    std::vector<uint32_t> act;
    const bool empty_window = d == 0 && c->win_wa == 0;  // a source shard without sources: no ingress words
    for (int64_t p = c->rl[d]; p < c->rh[d] && !empty_window; p++) {
      uint32_t i = I.of_pod[size_t(p)];
      if (!used[i]) {
        used[i] = 1;
        act.push_back(i);
      }
    }
    std::sort(act.begin(), act.end());
    {  // each active identity's first pod in the range: its plane row holds the class row in place
      std::vector<uint32_t> ar(I.ns.size(), 0xFFFFFFFFu);
      for (int64_t p = c->rh[d] - 1; p >= c->rl[d]; p--) ar[I.of_pod[size_t(p)]] = uint32_t(p - c->rl[d]);
      upload(c->arow[d], ar);
      c->n_act_ph1[d] = 0;  // (row phases: the phase-1 launch's representatives are among these)
      for (uint32_t i : act)
        if (c->phase_split && ar[i] < c->phase_split) c->n_act_ph1[d]++;
    }
    std::vector<uint8_t> ns_needed(pb.strings.size(), 0);
    for (uint32_t i : act) ns_needed[I.ns[i]] = 1;
    for (const DTarget& t : pb.tgt[d])
      if (ns_needed[t.ns])
        for (uint32_t j = t.poff; j < t.poff + t.pcnt; j++) peer_needed[j] = 1;
    c->n_act[d] = uint32_t(act.size());
    uint64_t tsum = 0;  // namespace targets each active identity's membership walk visits
    for (uint32_t i : act) tsum += pb.tns_hi[d][I.ns[i]] - pb.tns_lo[d][I.ns[i]];
    c->act_targets[d] = act.empty() ? 0.0 : double(tsum) / double(act.size());
    upload(c->act[d], act);
    // the membership's per-identity inputs in one 16-byte record (one load instead of the chain
    // act -> id_ls / id_ns / list_off -> tns_lo / tns_hi)
    std::vector<uint32_t> rec(act.size() * 4);
    for (size_t x = 0; x < act.size(); x++) {
      const uint32_t i = act[x], ns = I.ns[i];
      rec[4 * x] = I.ls[i];
      rec[4 * x + 1] = pb.tns_lo[d][ns];
      rec[4 * x + 2] = pb.tns_hi[d][ns];
      rec[4 * x + 3] = I.list_off[i];
    }
    upload(c->actrec[d], rec);
  }
  // selectors the range can reach: its targets' pod selectors and their peers' selectors
  std::vector<uint8_t> sel_needed(pb.S, 0);
  for (int d = 0; d < 2; d++)
    for (const DTarget& t : pb.tgt[d]) {
      bool needed = false;
      for (uint32_t j = t.poff; j < t.poff + t.pcnt && !needed; j++) needed = peer_needed[j];
      if (needed || t.pcnt == 0) sel_needed[t.sel] = 1;
    }
  for (int d = 0; d < 2; d++) {  // targets of active namespaces (also those without peers)
    const Identities& I = c->ids[d];
    std::vector<uint8_t> ns_needed(pb.strings.size(), 0);
    for (int64_t p = c->rl[d]; p < c->rh[d]; p++) ns_needed[I.ns[I.of_pod[size_t(p)]]] = 1;
    for (const DTarget& t : pb.tgt[d])
      if (ns_needed[t.ns]) sel_needed[t.sel] = 1;
  }
  for (uint32_t j = 0; j < pb.peers.size(); j++)
    if (peer_needed[j] && pb.peers[j].kind == PK_POD) {
      if (pb.peers[j].nskind == NS_LABEL) sel_needed[pb.peers[j].nsval] = 1;
      if (pb.peers[j].podsel != CYC_ALL) sel_needed[pb.peers[j].podsel] = 1;
    }
  std::vector<uint32_t> sl;
  for (uint32_t i = 0; i < pb.S; i++)
    if (sel_needed[i]) sl.push_back(i);
  c->n_sel = uint32_t(sl.size());
  {  // sparse pod rows: peers whose pod selector is one posting requirement are built from postings
    // (ingress peers first, then egress: each sub-list has its direction's word window)
    std::vector<uint32_t> scan, post;
    for (int d = 0; d < 2; d++) {
      c->scan_off[d] = uint32_t(scan.size());
      c->post_off[d] = uint32_t(post.size());
      for (uint32_t j : c->plan.pod_peers) {
        if (!peer_needed[j] || peer_dir[j] != d) continue;
        const DPeer& pr = pb.peers[j];
        if (pr.nskind == NS_ALL && pr.podsel == CYC_ALL) continue;  // all-ones row: the class rows need none
        const bool one = pr.podsel != CYC_ALL && pb.sel_off[pr.podsel + 1] - pb.sel_off[pr.podsel] == 1;
        if (one && c->dense_sel && !c->req_post_ok.empty() && c->req_post_ok[pb.sel_off[pr.podsel]]) post.push_back(j);
        else scan.push_back(j);
      }
    }
    c->scan_off[2] = uint32_t(scan.size());
    c->post_off[2] = uint32_t(post.size());
    c->n_scan = uint32_t(scan.size());
    c->n_post = uint32_t(post.size());
    upload(c->pp_scan, scan);
    upload(c->pp_post, post);
  }
  upload(c->sel_list, sl);
  std::vector<uint32_t> pp, ip;
  std::vector<DIPTest> tests;
  // An IP peer's row depends only on its IPBlock (ippeermatcher.go:43-50; the port is tested by the
  // class rows): peers of one direction whose (cidr, except) strings are equal share the row of
  // the first (config #4: the 0.0.0.0/0-style blocks of ~2,500 peers are 5 rows).  prow maps every
  // peer to its row; only the first of each IPBlock gets an IP-row test.
  std::vector<uint32_t> prow(std::max<size_t>(pb.peers.size(), 1));
  for (uint32_t j = 0; j < prow.size(); j++) prow[j] = j;
  std::vector<DIPRange> rtests;
  std::vector<uint2> riv;
  // an IPBlock's matching pods as intervals of the address index (its family's block, less each
  // same-family except), their count and word span: built from ranges when few and close
  // (no-panic runs only: the ordered walk with panic bits keeps its dense rows)
  const uint32_t n4 = uint32_t(c->ip4_key.size());
  // a network's pods of its family as positions [a, b) of the address index (ipsort_host)
  auto bounds = [&](const DCidr& cd, uint32_t& a, uint32_t& b) {
    if (cd.fam == 4) {
      const uint32_t lo = cd.net[3] & cd.mask[3], hi = lo | ~cd.mask[3];
      a = uint32_t(std::lower_bound(c->ip4_key.begin(), c->ip4_key.end(), lo) - c->ip4_key.begin());
      b = uint32_t(std::upper_bound(c->ip4_key.begin(), c->ip4_key.end(), hi) - c->ip4_key.begin());
    } else {
      std::array<uint32_t, 4> lo, hi;
      for (int i = 0; i < 4; i++) {
        lo[i] = cd.net[i] & cd.mask[i];
        hi[i] = lo[i] | ~cd.mask[i];
      }
      a = n4 + uint32_t(std::lower_bound(c->ip6_key.begin(), c->ip6_key.end(), lo) - c->ip6_key.begin());
      b = n4 + uint32_t(std::upper_bound(c->ip6_key.begin(), c->ip6_key.end(), hi) - c->ip6_key.begin());
    }
  };
  // ipaddress.go:22-40 on the index: the CIDR's positions less each same-family except's (an except of
  // the other family never contains a pod of this one); false if an except does not parse
  auto index_intervals = [&](const DIPTest& t, std::vector<uint2>& iv) -> bool {
    iv.assign(1, uint2{});
    bounds(t.cidr, iv[0].x, iv[0].y);
    for (uint32_t e = 0; e < t.excnt; e++) {
      const DCidr& x = c->plan.ip_ex[t.exoff + e];
      if (!x.valid) return false;
      if (x.fam != t.cidr.fam) continue;
      uint32_t ea, eb;
      bounds(x, ea, eb);
      std::vector<uint2> next;
      for (const uint2& v : iv) {
        if (ea > v.x) next.push_back(make_uint2(v.x, std::min(v.y, ea)));
        if (eb < v.y) next.push_back(make_uint2(std::max(v.x, eb), v.y));
      }
      iv.clear();
      for (const uint2& v : next)
        if (v.y > v.x) iv.push_back(v);
    }
    if (!iv.empty() && iv[0].y <= iv[0].x) iv.clear();  // a network holding no pod: no interval
    return true;
  };
  // IP rows as pod intervals: the family is address-monotone in pod order, so positions [a, b) of the
  // index are its pods ipsort_host[a] < ... < ipsort_host[b - 1] and nothing else of the family lies
  // between them: the row is the family's pods of pod indices [ipsort_host[a], ipsort_host[b - 1]]
  std::vector<DIPIv> vtests;
  std::vector<uint2> viv;
  auto iv_rows = [&](const DIPTest& t, DIPIv& out) -> bool {
    if (pb.may_err || !t.cidr.valid || c->ip_iv == 0 || !c->ip_mono[t.cidr.fam == 4 ? 0 : 1]) return false;
    std::vector<uint2> iv;
    if (!index_intervals(t, iv) || iv.size() > IPV_MAX) return false;
    out = DIPIv{t.peer, t.cidr.fam == 4 ? 0u : 1u, uint32_t(viv.size()), uint32_t(iv.size())};
    for (const uint2& v : iv) viv.push_back(make_uint2(c->ipsort_host[v.x], c->ipsort_host[v.y - 1] + 1));
    return true;
  };
  auto range_rows = [&](const DIPTest& t, DIPRange& out) -> bool {
    if (pb.may_err || !t.cidr.valid || c->ip_range == 0) return false;
    std::vector<uint2> iv;
    if (!index_intervals(t, iv)) return false;
    uint64_t n = 0;
    for (const uint2& v : iv) n += v.y - v.x;
    if (n > IPR_MAX_MATCH) return false;
    uint32_t wlo = 0xFFFFFFFFu, whi = 0;
    for (const uint2& v : iv)
      for (uint32_t x = v.x; x < v.y; x++) {
        wlo = std::min(wlo, c->ipsort_host[x] / 64);
        whi = std::max(whi, c->ipsort_host[x] / 64);
      }
    if (n && whi - wlo >= IPR_SPAN) return false;
    // words whose pods of the family hold affine addresses get the network's lanes from its bounds
    // in k_ip_rows_fast (no per-pod test): keep those rows there (config #4: range-built rows
    // made launch B 64 -> 70 us; config #2's addresses step by 256, so its words are not affine)
    const uint8_t fbit = t.cidr.fam == 4 ? 1u : 2u;
    bool all_aff = c->word_aff.size() == pb.W;
    for (uint32_t w = wlo; all_aff && n && w <= whi; w++) all_aff = (c->word_aff[w] & fbit) != 0;
    if (all_aff && c->ip_range < 0) return false;
    out = DIPRange{t.peer, uint32_t(riv.size()), uint32_t(iv.size()), n ? wlo : 0u};
    riv.insert(riv.end(), iv.begin(), iv.end());
    return true;
  };
  for (int d = 0; d < 2; d++) {  // ingress peers first, then egress: one sub-list per branch
    c->rp_off[d] = uint32_t(pp.size());
    c->ri_off[d] = uint32_t(ip.size());
    c->rr_off[d] = uint32_t(rtests.size());
    c->rv_off[d] = uint32_t(vtests.size());
    for (uint32_t j : c->plan.pod_peers)
      if (peer_needed[j] && peer_dir[j] == d) pp.push_back(j);
    std::map<std::vector<uint32_t>, uint32_t> ipb_row;
    std::vector<uint32_t> key;
    for (size_t r = 0; r < c->plan.ip_peers.size(); r++) {
      const uint32_t j = c->plan.ip_peers[r];
      if (!peer_needed[j] || peer_dir[j] != d) continue;
      const DIPBlock& b = pb.ipbs[pb.peers[j].ipb];
      key.assign(1, b.cidr);
      key.insert(key.end(), pb.ipb_ex.begin() + b.exoff, pb.ipb_ex.begin() + b.exoff + b.excnt);
      auto it = ipb_row.emplace(key, j);
      if (!it.second) {
        prow[j] = it.first->second;
        continue;
      }
      DIPIv vt{};
      if (iv_rows(c->plan.ip_tests[r], vt)) {
        vtests.push_back(vt);
        continue;
      }
      DIPRange rt{};
      if (range_rows(c->plan.ip_tests[r], rt)) {
        rtests.push_back(rt);
        continue;
      }
      ip.push_back(j);
      tests.push_back(c->plan.ip_tests[r]);
    }
  }
  c->rr_off[2] = uint32_t(rtests.size());
  c->Rr = uint32_t(rtests.size());
  upload(c->ipr_tests, rtests);
  upload(c->ipr_iv, riv);
  c->rv_off[2] = uint32_t(vtests.size());
  c->Rv = uint32_t(vtests.size());
  upload(c->ipv_tests, vtests);
  upload(c->ipv_iv, viv);
  upload(c->peer_row, prow);
  c->prow_host = prow;
  c->rp_off[2] = uint32_t(pp.size());
  c->ri_off[2] = uint32_t(ip.size());
  c->Rp = uint32_t(pp.size());
  c->Ri = uint32_t(ip.size());
  upload(c->pod_peers, pp);
  {
    // IDOB rows depend on a pod peer only through (namespace matcher, pod selector)
    // (podpeermatcher.go:21-28; the port is checked per peer by the class rows), so peers sharing
    // them share one row: config #3 has 17k pod peers over 7.8k distinct matchers
    // The rows are ordered exact-namespace matchers first, by namespace, so a group of PB_GROUP rows
    // mostly names one or two namespaces: its identity-set waves over words of other namespaces'
    // identities skip every selector (grp_ns / word_ns below).
    std::vector<uint32_t> pi(std::max<size_t>(pb.peers.size(), 1), 0), ppu;
    std::vector<uint2> gns;
    for (int d = 0; d < 2; d++) {
      c->rpu_off[d] = uint32_t(ppu.size());
      c->ido_goff[d] = uint32_t(gns.size());
      std::map<std::tuple<uint32_t, uint32_t, uint32_t>, uint32_t> row;  // matcher -> its first peer
      for (uint32_t x = c->rp_off[d]; x < c->rp_off[d + 1]; x++) {
        const DPeer& pr = pb.peers[pp[x]];
        row.emplace(std::make_tuple(pr.nskind, pr.nsval, pr.podsel), pp[x]);
      }
      const uint32_t u0 = uint32_t(ppu.size());
      std::map<std::tuple<uint32_t, uint32_t, uint32_t>, uint32_t> at;
      for (const auto& kv : row) {  // (nskind 0 = exact namespace sorts first, then by namespace)
        at[kv.first] = uint32_t(ppu.size());
        ppu.push_back(kv.second);
      }
      for (uint32_t x = c->rp_off[d]; x < c->rp_off[d + 1]; x++) {
        const DPeer& pr = pb.peers[pp[x]];
        pi[pp[x]] = at[std::make_tuple(pr.nskind, pr.nsval, pr.podsel)];
      }
      for (uint32_t g0 = u0; g0 < ppu.size(); g0 += PB_GROUP) {
        uint2 r{0xFFFFFFFFu, 0u};
        for (uint32_t x = g0; x < std::min<uint32_t>(g0 + PB_GROUP, uint32_t(ppu.size())); x++) {
          const DPeer& pr = pb.peers[ppu[x]];
          if (pr.nskind != 0) r = uint2{0u, 0xFFFFFFFFu};  // a namespace / all-namespace matcher: never skipped
          if (r.x == 0 && r.y == 0xFFFFFFFFu) break;
          r.x = std::min(r.x, pr.nsval);
          r.y = std::max(r.y, pr.nsval);
        }
        gns.push_back(r);
      }
    }
    c->rpu_off[2] = uint32_t(ppu.size());
    upload(c->pod_peers_u, ppu);
    {  // the rows' matcher records (pb_rec), read by the identity-set waves when selectors are evaluated there
      std::vector<uint4> rec(std::max<size_t>(ppu.size(), 1) * 3, uint4{0, 0, 0, 0});
      const bool one = c->sel_one_h.size() >= std::max<size_t>(pb.S, 1);
      for (size_t x = 0; one && x < ppu.size(); x++) {
        const DPeer& pr = pb.peers[ppu[x]];
        rec[3 * x] = uint4{pr.nskind, pr.nsval, pr.podsel, 0u};
        rec[3 * x + 1] = pr.nskind == 2 ? c->sel_one_h[pr.nsval] : uint4{SEL_ALL, 0u, 0u, 0u};
        rec[3 * x + 2] = pr.podsel != CYC_ALL ? c->sel_one_h[pr.podsel] : uint4{SEL_ALL, 0u, 0u, 0u};
      }
      if (one) upload(c->pb_rec, rec);
      else c->pb_rec.alloc(0);
    }
    upload(c->peer_ido, pi);
    gns.push_back(uint2{0u, 0xFFFFFFFFu});
    upload(c->ido_grp_ns, gns);
    const auto& ins = c->ids[1].ns;  // egress identities' namespaces, per 64-identity word
    std::vector<uint2> wns(std::max<size_t>((ins.size() + 63) / 64, 1), uint2{0xFFFFFFFFu, 0u});
    for (size_t e = 0; e < ins.size(); e++) {
      wns[e / 64].x = std::min(wns[e / 64].x, ins[e]);
      wns[e / 64].y = std::max(wns[e / 64].y, ins[e]);
    }
    upload(c->ido_word_ns, wns);
  }
  upload(c->ip_peers, ip);
  upload(c->ip_tests, tests);
  upload(c->ip_ex, c->plan.ip_ex);
  {  // IP-row work items of the fused front's segments (ip_rows_items_blk): per chunk of a segment's
     // window, its rows whose network meets the chunk's addresses (the chunk test of
     // ip_rows_fast_blk), IPI_TOUCH to a wave, and the others 64 to a wave (their chunk flags cleared)
    std::vector<DIPItem> items;
    std::vector<uint32_t> il;
    const bool one = one_window(c);
    const uint32_t NCH = (pb.W + 63) / 64;
    // auto: whole-table runs only — a shard's few IP rows and windows ran launch B 2x slower as items
    // (config #3 rank 0 of 8: B 45.5 vs 20.9 us source, 36.4 vs 17.0 target; whole step +20 us), while
    // whole tables gain 0-1 % (profiles/r05_ip_items_ab.txt)
    const bool whole = lo == 0 && hi == int64_t(pb.P);
    const bool on = (c->ip_items_opt == 1 || (c->ip_items_opt == -1 && whole)) && c->ipw_h.size() == size_t(pb.W) + NCH &&
                    !pb.may_err;
    for (int x = 0; x < 2; x++) {
      c->ipi_off[x] = uint32_t(items.size());
      if (!on || (one && x)) continue;
      const int dlo = one ? 0 : x, dhi = one ? 2 : x + 1;
      const uint32_t i0 = c->ri_off[dlo], n = c->ri_off[dhi] - i0;
      uint32_t c0, nch;
      peer_chunks(c, one ? 1 : x, c0, nch);
      std::vector<uint32_t> hit, miss;
      for (uint32_t ch = c0; n && ch < c0 + nch; ch++) {
        const DWordIP& ck = c->ipw_h[pb.W + ch];
        hit.clear();
        miss.clear();
        for (uint32_t r = 0; r < n; r++) (ip_chunk_touch(tests[i0 + r].cidr, ck) ? hit : miss).push_back(r);
        for (const auto* v : {&hit, &miss}) {
          const uint32_t per = v == &hit ? IPI_TOUCH : 64u;
          for (size_t a = 0; a < v->size(); a += per) {
            const uint32_t cnt = uint32_t(std::min<size_t>(per, v->size() - a));
            items.push_back(DIPItem{ch, uint32_t(il.size()), cnt, v == &hit ? 1u : 0u});
            il.insert(il.end(), v->begin() + a, v->begin() + a + cnt);
          }
        }
      }
    }
    c->ipi_off[2] = uint32_t(items.size());
    c->ip_items = on && !items.empty();
    upload(c->ipi_items, items);
    upload(c->ipi_list, il);
  }
  clk.lap("done");
  c->order_lo = lo;
  c->order_hi = hi;
  c->order_src = src;
}

// Word window of direction d's peer rows in the current plan: [w0, w0 + nw); as 64-word chunks
// [c0, c0 + nch).
static void peer_window(const cyc_ctx* c, int d, uint32_t& w0, uint32_t& nw) {
  w0 = d == 0 ? c->win_w0 : 0u;
  nw = d == 0 ? c->win_wa : c->pb.W;
}
static void peer_chunks(const cyc_ctx* c, int d, uint32_t& c0, uint32_t& nch) {
  uint32_t w0, nw;
  peer_window(c, d, w0, nw);
  c0 = w0 / 64;
  nch = nw ? (w0 + nw + 63) / 64 - c0 : 0u;
}
// the two directions' peer rows share one window (target-row plans): one launch segment for both
static bool one_window(const cyc_ctx* c) { return c->win_w0 == 0 && c->win_wa == c->pb.W; }
