// enqueue.hpp — enqueueing a run: the pipeline pieces, the fused front, the emit, graph capture and replay.
// Part of engine.hip's single translation unit (device bodies inline across stages, host helpers are
// static): included once, by engine.hip, in stage order.
#pragma once

// Pipeline pieces.  Steps 1, 3, 4 are shared; steps 2 and 5-7 run per direction (ingress peers,
// targets, class rows and plane are disjoint from egress ones), so the two directions can run
// as two independent branches: one direction's front hides under the other's HBM-bound emit.
enum { COMMON_SELECTORS = 1, COMMON_PORTS = 2, COMMON_FILL = 4, COMMON_ALL = 7 };
// Descriptor bit rows of the port table for the egress class rows (cyc_set_option "port_bits")
static bool port_bits_on(const cyc_ctx* c) { return std::max<size_t>(c->pb.descs.size(), 1) <= 32; }

static void enq_common(cyc_ctx* c, hipStream_t st, int parts = COMMON_ALL) {
  Problem& pb = c->pb;
  const uint32_t P = pb.P, K = pb.K, W = pb.W, D = uint32_t(std::max<size_t>(pb.descs.size(), 1));
  const uint32_t M = uint32_t(pb.pms.size());
  if ((parts & COMMON_FILL) && !pb.may_err && (c->Ri || c->Rr))  // IP-peer word spans (k_ip_rows_fast)
    k_fill_u32<<<grid1(c->pb.peers.size() * 4, 256), 256, 0, st>>>(c->ip_rng.as<uint32_t>(), c->pb.peers.size() * 4, 0xFFFFFFFFu);
  if (!(parts & COMMON_SELECTORS)) goto ports;
  // 1. selectors x label sets
  if (uint64_t(c->n_sel) * pb.L && c->dense_sel)
    k_selectors_dense<<<unsigned(uint64_t(c->n_sel) * ((pb.L + 256 * SEL_LPT - 1) / (256 * SEL_LPT))), 256, 0, st>>>(
        c->n_sel, pb.L, c->sel_off.as<uint32_t>(), c->dreqs.as<DReq>(), c->req_vals.as<uint32_t>(), c->lvt.as<uint32_t>(),
        c->selres.as<uint8_t>(), c->sel_list.as<uint32_t>());
  else if (uint64_t(c->n_sel) * pb.L)
    k_selectors<<<grid1(uint64_t(c->n_sel) * pb.L, 256), 256, 0, st>>>(
        c->n_sel, pb.L, c->sel_off.as<uint32_t>(), c->reqs.as<DReq>(), c->req_vals.as<uint32_t>(), c->ls_off.as<uint32_t>(),
        c->ls_key.as<uint32_t>(), c->ls_val.as<uint32_t>(), c->selres.as<uint8_t>(), c->sel_list.as<uint32_t>());
ports:
  if (!(parts & COMMON_PORTS)) return;
  // 3. port matchers x job descriptors
  if (M && pb.descs.size())
    k_portok<<<grid1(uint64_t(M) * D, 256), 256, 0, st>>>(M, D, c->pms.as<DPortM>(), c->pents.as<DPortEntry>(),
                                                          c->descs.as<DDesc>(), c->portok.as<uint8_t>());
  if (M && pb.descs.size() && port_bits_on(c))
    k_portbits<<<(M + 255) / 256, 256, 0, st>>>(M, D, c->portok.as<uint8_t>(), c->portbits.as<uint32_t>());
  // 4. per-slot destination words
  if (uint64_t(K) * W)
    k_slot_words<<<unsigned((uint64_t(K) * W + 3) / 4), 256, 0, st>>>(
        P, K, W, D, c->slot_desc.as<int32_t>(), c->slot_status.as<uint8_t>(), c->VALID.as<uint64_t>(),
        c->DESCW.as<int32_t>(), c->DM.as<uint64_t>());
}

// Pod peers folded into per-class identity sets, expanded by the class rows over each word's
// identity runs (no PM pod rows)?  Needs: no panic possible (the panic path walks PM / ER rows in
// peer order), few runs per word, and identity sets of bounded size.
static bool ido_mode(const cyc_ctx* c) { return c->pod_words != 0 && c->pb.blocks.empty() && ido_possible(c); }

// 2. peer rows of direction d's peers: pod peers in identity space, expanded over word runs
// (skipped in IDO mode: the class rows expand them); IP peers per pod
enum { PEERS_POD = 1, PEERS_IP = 2 };
static void enq_peer_rows(cyc_ctx* c, int d, hipStream_t st, int which = PEERS_POD | PEERS_IP) {
  Problem& pb = c->pb;
  const uint32_t P = pb.P, W = pb.W;
  const uint32_t E = c->dir[1].n;
  // d = 2: both directions in one launch (their peer sub-lists are adjacent) when they share a window
  if (d == 2 && !one_window(c)) {
    enq_peer_rows(c, 0, st, which);
    enq_peer_rows(c, 1, st, which);
    return;
  }
  const int dlo = d == 2 ? 0 : d, dhi = d == 2 ? 2 : d + 1;
  uint32_t w0, nw, c0, nch;  // the rows' word window (a source shard's ingress peers: its sources' words)
  peer_window(c, d == 2 ? 1 : d, w0, nw);
  peer_chunks(c, d == 2 ? 1 : d, c0, nch);
  const uint32_t r0 = c->rp_off[dlo], Rp = (which & PEERS_POD) ? c->rp_off[dhi] - r0 : 0u;
  if (Rp && E && W && ido_mode(c)) {
    const uint32_t EW = (E + 63) / 64;
    for (int x = dlo; x < dhi; x++) {  // per direction: its identity word window
      const uint32_t u0 = c->rpu_off[x], Ru = c->rpu_off[x + 1] - u0;  // distinct matchers only
      const uint32_t ew0 = x == 0 ? c->ido_ew0 : 0u, new_ = x == 0 ? c->ido_ew1 - c->ido_ew0 : EW;
      if (Ru && new_)
        k_peer_bits<<<unsigned((uint64_t((Ru + PB_GROUP - 1) / PB_GROUP) * new_ + 3) / 4), 256, 0, st>>>(
            Ru, E, EW, c->pod_peers_u.as<uint32_t>() + u0, c->peers.as<DPeer>(), c->selres.as<uint8_t>(), pb.L,
            c->dir[1].id_ns.as<uint32_t>(), c->id_nsls.as<uint32_t>(), c->dir[1].id_ls.as<uint32_t>(),
            c->idob.as<uint64_t>() + uint64_t(u0) * EW, ew0, new_, c->ido_grp_ns.as<uint2>() + c->ido_goff[x],
            c->ido_word_ns.as<uint2>());
    }
  } else if (Rp && E && nw && (c->pod_rows >= 0 ? c->pod_rows == 1 : uint64_t(E) * 2 >= P)) {
    const uint32_t* plist = c->pod_peers.as<uint32_t>() + r0;
    const unsigned g = unsigned((pod_direct_waves(Rp, nw) + 3) / 4);
    const uint32_t* eid = c->dir[1].pod_id.as<uint32_t>();
    if (pb.may_err)
      k_pod_rows_direct<true><<<g, 256, 0, st>>>(Rp, P, W, plist, c->peers.as<DPeer>(), c->selres.as<uint8_t>(), pb.L, eid,
                                                 c->dir[1].id_ns.as<uint32_t>(), c->id_nsls.as<uint32_t>(),
                                                 c->dir[1].id_ls.as<uint32_t>(), c->PM.as<uint64_t>(), c->ER.as<uint64_t>(), w0, nw);
    else
      k_pod_rows_direct<false><<<g, 256, 0, st>>>(Rp, P, W, plist, c->peers.as<DPeer>(), c->selres.as<uint8_t>(), pb.L, eid,
                                                  c->dir[1].id_ns.as<uint32_t>(), c->id_nsls.as<uint32_t>(),
                                                  c->dir[1].id_ls.as<uint32_t>(), c->PM.as<uint64_t>(), c->ER.as<uint64_t>(), w0, nw);
  } else if (Rp && E && nw) {
    const uint32_t* plist = c->pod_peers.as<uint32_t>() + r0;
    uint8_t* ido = c->ido.as<uint8_t>() + uint64_t(r0) * E;
    k_peer_ident<<<grid1(uint64_t(Rp) * E, 256), 256, 0, st>>>(Rp, E, plist, c->peers.as<DPeer>(), c->selres.as<uint8_t>(),
                                                               pb.L, c->dir[1].id_ns.as<uint32_t>(),
                                                               c->id_nsls.as<uint32_t>(), c->dir[1].id_ls.as<uint32_t>(), ido);
    unsigned g = unsigned(uint64_t((nw + 255) / 256) * Rp);
    if (pb.may_err)
      k_pod_rows<true><<<g, 256, 0, st>>>(Rp, E, W, plist, ido, c->word_off.as<uint32_t>(), c->run_e.as<uint32_t>(),
                                          c->run_mask.as<uint64_t>(), c->PM.as<uint64_t>(), c->ER.as<uint64_t>(), w0, nw);
    else
      k_pod_rows<false><<<g, 256, 0, st>>>(Rp, E, W, plist, ido, c->word_off.as<uint32_t>(), c->run_e.as<uint32_t>(),
                                           c->run_mask.as<uint64_t>(), c->PM.as<uint64_t>(), c->ER.as<uint64_t>(), w0, nw);
  }
  const uint32_t v0 = c->rv_off[dlo], Rv = (which & PEERS_IP) ? c->rv_off[dhi] - v0 : 0u;
  if (Rv && nw)
    k_ip_rows_iv<<<(Rv + 3) / 4, 256, 0, st>>>(Rv, W, c->ipv_tests.as<DIPIv>() + v0, c->ipv_iv.as<uint2>(),
                                             c->ip_words.as<DWordIP>(), c->PM.as<uint64_t>(), c->ip_rng.as<uint32_t>(), ip_cnz(c),
                                             c0, nch);
  const uint32_t q0 = c->rr_off[dlo], Rr = (which & PEERS_IP) ? c->rr_off[dhi] - q0 : 0u;
  if (Rr && nw)
    k_ip_rows_range<<<(Rr + 3) / 4, 256, 0, st>>>(Rr, W, c->ipr_tests.as<DIPRange>() + q0, c->ipr_iv.as<uint2>(),
                                                c->ipsort.as<uint32_t>(), c->PM.as<uint64_t>(), c->ip_rng.as<uint32_t>(), ip_cnz(c), c0, nch);
  const uint32_t i0 = c->ri_off[dlo], Ri = (which & PEERS_IP) ? c->ri_off[dhi] - i0 : 0u;
  if (Ri && nw) {
    const DIPTest* tests = c->ip_tests.as<DIPTest>() + i0;
    if (pb.may_err) {
      // batch size: as many peers per block as keep >= ~2048 blocks in flight, at most IPB_BATCH
      const uint64_t wch = (nw + 3) / 4;
      const uint64_t nb_want = (2048 + wch - 1) / wch;
      const uint32_t bat = uint32_t(std::max<uint64_t>(1, std::min<uint64_t>(IPB_BATCH, (Ri + nb_want - 1) / nb_want)));
      unsigned g = unsigned(wch * ((Ri + bat - 1) / bat));
      k_ip_rows<true><<<g, 256, 0, st>>>(Ri, P, W, tests, c->ip_ex.as<DCidr>(), c->pod_ip.as<DIP>(), c->PM.as<uint64_t>(),
                                         c->ER.as<uint64_t>(), bat, w0, nw);
    } else {
      const uint32_t grp = IP_GROUP;
      k_ip_rows_fast<<<unsigned(ip_rows_blocks(Ri, nch, grp)), 256, 0, st>>>(
          Ri, P, W, tests, c->ip_ex.as<DCidr>(), c->pod_ip.as<DIP>(), c->ip_words.as<DWordIP>(), c->PM.as<uint64_t>(),
          c->ip_rng.as<uint32_t>(), ip_cnz(c), grp, c0, nch);
    }
  }
}

// 5. membership + classes of direction d
static void enq_member_clear(cyc_ctx* c, int d, hipStream_t st) {
  DirDev& dd = c->dir[d];
  if (dd.n) HIPCHK(hipMemsetAsync(dd.ht_key.p, 0xFF, dd.ht_key.bytes, st));  // keys and reps: one buffer
}

// The class rows of a run empty the hash table for the next one (ht_clear_slice); only runs whose
// class rows do not launch (no slots or no pods) need the memset (prepare_device empties it once).
static bool class_rows_clear_ht(const cyc_ctx* c, int d) {
  return c->dir[d].n && c->pb.K && c->pb.W && c->n_act[d];
}

static void enq_member(cyc_ctx* c, int d, hipStream_t st, bool clear = true) {
  DirDev& dd = c->dir[d];
  if (!dd.n) return;
  if (clear && !class_rows_clear_ht(c, d)) enq_member_clear(c, d, st);
  MemberArgs ma = member_args(c, d);
  if (!c->n_act[d]) return;
  // auto (-1): a wave per identity while identities are few (<= 4096) and each walks several
  // targets (>= 4 on average): config #3 (2000 identities, ~6 targets each) gains, configs #2
  // (10k identities), #4 (38k) and #5 (~0.3 targets each) lose (profiles/r01_member_wave_ab.txt)
  if (c->member_wave > 0 || (c->member_wave < 0 && c->n_act[d] <= 4096 && c->act_targets[d] >= 4.0)) k_member_wave<<<unsigned((uint64_t(c->n_act[d]) + 3) / 4), 256, 0, st>>>(ma);
  else k_member<<<grid1(c->n_act[d], 128), 128, 0, st>>>(ma);
  k_classify<<<grid1(c->n_act[d], 256), 256, 0, st>>>(ma, dd.class_of.as<uint32_t>());
}

#ifndef CYC_PHASE_GRID
#define CYC_PHASE_GRID 1  // row phases: each class-row launch's grid sized by its phase's identities (0: all)
#endif
#ifndef CYC_PB_REC
#define CYC_PB_REC 1  // identity-set waves read their rows' matcher records (pb_rec); 0: the peers' chains
#endif

// 6. class rows of direction d
// IDO class rows: representatives per block (cyc_set_option "class_rpb"; 0 = auto: 4, or more in
// the fused front, enq_front_fused), as many as fit the staged identity-set budget
static uint32_t class_rpb(const cyc_ctx* c, size_t per_rep_lds, uint32_t want = 0) {
  const uint64_t fit = std::max<uint64_t>(1, IDO_LDS_BYTES / std::max<size_t>(per_rep_lds, 1));
  const int64_t w = want ? int64_t(want) : c->class_rpb_opt ? c->class_rpb_opt : 4;
  return uint32_t(std::max<int64_t>(1, std::min<int64_t>(w, int64_t(fit))));
}

static RowArgs row_args(cyc_ctx* c, int d) {
  Problem& pb = c->pb;
  const uint32_t P = pb.P, K = pb.K, W = pb.W, D = uint32_t(std::max<size_t>(pb.descs.size(), 1));
  DirDev& dd = c->dir[d];
  RowArgs ra{};
  ra.tgt = dd.tgt.as<DTarget>();
  ra.peers = c->peers.as<DPeer>();
  ra.PM = c->PM.as<uint64_t>();
  ra.ER = c->ER.as<uint64_t>();
  ra.portok = c->portok.as<uint8_t>();
  // descriptor bit rows of the port table (k_portbits; computed whenever D <= 32)
  ra.portbits = port_bits_on(c) && pb.pms.size() && pb.descs.size() ? c->portbits.as<uint32_t>() : nullptr;
  ra.D = D;
  ra.n_ident = dd.n;
  ra.K = K;
  ra.W = W;
  ra.P = P;
  peer_window(c, d, ra.w0, ra.WA);  // the class rows cover their peers' word window
  if (!c->pb.blocks.empty()) {     // batched blocks: each class row covers its block's words
    ra.w0 = 0;
    ra.WA = c->blk_wa_max;
    ra.id_win = c->id_win[d].as<uint2>();
  }
  ra.class_of = dd.class_of.as<uint32_t>();
  ra.cnt = dd.cnt.as<uint32_t>();
  ra.list_off = dd.list_off.as<uint32_t>();
  ra.list = dd.list.as<uint32_t>();
  ra.id_err = dd.err.as<uint8_t>();
  ra.id_desc = dd.id_desc.as<int32_t>();
  ra.id_status = dd.id_status.as<uint8_t>();
  ra.VALID = c->VALID.as<uint64_t>();
  ra.DESCW = c->DESCW.as<int32_t>();
  ra.DM = c->DM.as<uint64_t>();
  ra.A = dd.A.as<uint64_t>();
  ra.AE = pb.may_err ? dd.AE.as<uint64_t>() : nullptr;
  ra.rep_blocks = c->n_act[d];  // k_class_rows (panic path): a block row per representative slot
  ra.reps = dd.reps.as<uint32_t>();
  ra.rep_cnt = dd.rep_cnt();
  ra.IDOB = c->idob.as<uint64_t>();
  ra.peer_ido = c->peer_ido.as<uint32_t>();
  ra.prow = c->peer_row.as<uint32_t>();
  ra.zero = c->zeros.as<uint64_t>();
  ra.runs = c->runs.as<WordRuns>();
  ra.B = dd.B.as<uint64_t>();
  ra.ip_off = dd.ip_off.as<uint32_t>();
  ra.ip_cnt = dd.ip_cnt.as<uint32_t>();
  ra.ip_list = dd.ip_list.as<uint4>();
  ra.ip_rng = c->ip_rng.as<uint32_t>();
  ra.ip_cnz = ip_cnz(c);
  ra.E = c->dir[1].n;
  ra.EW = (ra.E + 63) / 64;
  ra.ew_lo = d == 0 ? c->ido_ew0 : 0u;
  ra.ew_hi = d == 0 ? c->ido_ew1 : ra.EW;
  ra.NB = d == 0 ? K : D;
  // the first kernel below empties the hash table for the next run (keys + reps; not the counter)
  ra.ht_clear = reinterpret_cast<uint32_t*>(dd.ht_key.p);
  ra.ht_clear_words = uint64_t(dd.ht_cap) * 4;
  ra.rpb = 1;
  return ra;
}

// PM-build class rows a wave per 64-word chunk (pl_wave_chunks): both directions' accumulators fit
// (descriptors and slots <= PL_NB) and every peer's port bits are available.
static bool pl_wave_ok(const cyc_ctx* c) {
  const Problem& pb = c->pb;
  return c->pl_wave && pb.K <= PL_NB && pb.descs.size() <= PL_NB && pb.descs.size() && pb.pms.size() &&
         port_bits_on(c) && pb.W <= 64 * 64;
}

static void enq_class_rows(cyc_ctx* c, int d, hipStream_t st) {
  Problem& pb = c->pb;
  const uint32_t K = pb.K, W = pb.W, D = uint32_t(std::max<size_t>(pb.descs.size(), 1));
  DirDev& dd = c->dir[d];
  if (!dd.n || !K || !W || !c->n_act[d]) return;
  RowArgs ra = row_args(c, d);
  if (!ra.WA) return;
  if (pb.may_err) {  // the ordered walk with panic bits: one block row per identity, 8 slots per thread
    const unsigned g = unsigned(uint64_t((ra.WA + 255) / 256) * ((K + 7) / 8) * ra.rep_blocks);
    if (d == 0) k_class_rows<false><<<g, 256, 0, st>>>(ra);
    else k_class_rows<true><<<g, 256, 0, st>>>(ra);
  } else if (ido_mode(c)) {
    // identity sets first (one wave per representative and 4 slots / descriptors), then the rows
    const uint64_t waves = uint64_t(c->n_act[d]) * ((ra.NB + CI_G - 1) / CI_G);
    if (d == 0) k_class_ident<false, CI_G><<<unsigned((waves + 3) / 4), 256, 0, st>>>(ra);
    else k_class_ident<true, CI_G><<<unsigned((waves + 3) / 4), 256, 0, st>>>(ra);
    ra.ht_clear_words = 0;
    const uint32_t rows = d == 0 ? 4u : D;  // (class_rows_ido_blk stages KC = 4 slot rows, or D descriptor rows)
    const size_t per = size_t(rows) * ra.EW * 8 + IDO_IPL * sizeof(uint4) + 16;  // identity sets + staged IP peers (+ alignment)
    ra.rpb = class_rpb(c, per);
    const unsigned gi = unsigned(uint64_t(ido_chunk_groups(ra.WA)) * ((K + 3) / 4) * ((c->n_act[d] + ra.rpb - 1) / ra.rpb));
    if (d == 0) k_class_rows_ido<false, 4><<<gi, 256, per * ra.rpb, st>>>(ra);
    else k_class_rows_ido<true, 4><<<gi, 256, per * ra.rpb, st>>>(ra);
  } else {  // per-class flattened peer lists (the IP word spans are final here)
    const bool wave = pl_wave_ok(c);
    if (d == 0 && wave) k_class_rows_pl<false, true><<<pl_blocks(c, d), pl_threads(c), 0, st>>>(ra);
    else if (d == 0) k_class_rows_pl<false, false><<<pl_blocks(c, d), pl_threads(c), 0, st>>>(ra);
    else if (wave) k_class_rows_pl<true, true><<<pl_blocks(c, d), pl_threads(c), 0, st>>>(ra);
    else k_class_rows_pl<true, false><<<pl_blocks(c, d), pl_threads(c), 0, st>>>(ra);
  }
}

// 7. the emit: both planes (ingress rows to out_in, egress rows to out_eg) in one launch — two
// when their rows differ in length (a source shard: ingress rows of every destination over the
// shard's word window, egress rows of its sources over all words).  d_status (may be null): the
// status plane, copied by the (first) emit's blocks.  Returns false if no emit was launched (no rows
// in the plan; the caller then copies the status plane itself).
constexpr uint64_t EMIT_WIDE_MIN = 16384;  // shortest plane row (bytes) emitted a block per row; shorter: k_emit_flat
// k_emit_units over ea.n_rows[] rows of ea.pl_words[] words per plane (16-byte aligned planes, even
// row words): units of about one 1024 x 7 x 16 B block pass (114 KB) — whole rows of up to that, or
// several shorter rows — so a block resolves its rows' order -> identity -> class chains together
static const char* enq_emit_units(EmitArgs ea, hipStream_t st) {
  constexpr uint64_t pass = 1024 * 7 * 16;
  for (int pl = 0; pl < 2; pl++) {
    const uint64_t rb = std::max<uint64_t>(ea.pl_words[pl] * 8, 1);
    ea.unit_rows[pl] = uint32_t(std::min<uint64_t>(EMIT_UNIT_MAX_ROWS, std::max<uint64_t>(1, pass / rb)));
    // rows of 7-14 KB (a source shard's ingress rows at N = 8: 12.5 KB) as 8 rows a unit, a row per
    // 128-thread group in one aligned buffer-op pass: config #3 rank 0 of 8 emit 384 vs 425 us, step
    // -3 %; 512- and 256-thread groups for the 50 / 25 KB rows of N = 2 / 4 measured +1 % / ±0: not
    // used (profiles/r05_row_alignment.txt)
    ea.unit_grp[pl] = 0;
    if (rb <= pass / 8 && rb > pass / 16 && rb % 16 == 0) {
      ea.unit_grp[pl] = 8;
      ea.unit_rows[pl] = 8;
    }
    ea.n_units[pl] = (ea.n_rows[pl] + ea.unit_rows[pl] - 1) / ea.unit_rows[pl];
  }
  ea.per_xcd = (ea.n_units[0] + ea.n_units[1] + 7) / 8;
  k_emit_units<1024, 7><<<ea.per_xcd * 8, 1024, 0, st>>>(ea);
  return "k_emit_units<1024,7>";
}


static const char* enq_emit_launch(const EmitArgs& ea_in, hipStream_t st, uint64_t* out_in, uint64_t* out_eg) {
  EmitArgs ea = ea_in;
  const uint32_t nr = ea.n_rows[0] + ea.n_rows[1];
  ea.per_xcd = (nr + 7) / 8;
  const bool aligned = reinterpret_cast<uintptr_t>(out_in) % 16 == 0 && reinterpret_cast<uintptr_t>(out_eg) % 16 == 0;
  const unsigned g = ea.per_xcd * 8;  // one block per row slot of the 8 XCD segments
  if (ea.row_words % 2 || !aligned) {
    k_emit_words<<<g, 256, 0, st>>>(ea);
    return "k_emit_words";
  }
  const uint64_t row_bytes = ea.row_words * 8;
  // 56-112 KB rows (config #3's 98 KB): 1024 x 7 blocks through buffer ops, one pass.  A 512 x 13
  // one-pass block held 84 VGPRs with flat addresses (config #3 3.5 % slower, profiles/r03_emit_ab.txt)
  // and 54 through buffer ops, 1-2 % ahead of 1024 x 7 on the best plane placements but up to 20 %
  // behind on others: over 14 placements 3.542 vs 3.389 ms per step (profiles/r05_plane_placement.txt;
  // the flat-address 1024 x 7 form trailed both) — only 1024 x 7 through buffer ops is kept.
  // (128 x 13 buffer blocks for config #4's 25 KB rows lost: 442-447 vs 419-424 us.)
  if (row_bytes > 512 * 7 * 16 && row_bytes <= 1024 * 7 * 16) {
    k_emit_wide_buf<1024, 7><<<g, 1024, 0, st>>>(ea);
    return "k_emit_wide_buf<1024,7>";
  } else if (row_bytes > 512 * 7 * 16) {  // > 104 KB: 1024 x 7 passes
    k_emit_wide<1024, 7><<<g, 1024, 0, st>>>(ea);
    return "k_emit_wide<1024,7>";
  } else if (row_bytes > 256 * 8 * 16) {  // 32-56 KB: 512 x 7 (source shards at N = 2)
    k_emit_wide<512, 7><<<g, 512, 0, st>>>(ea);
    return "k_emit_wide<512,7>";
  } else if (row_bytes >= EMIT_WIDE_MIN) {  // 256-thread single pass (16-32 KB rows; buffer-op 256 x 8,
                                            // 512 x 4 and 1024 x 2 blocks were no better over 4 plane
                                            // placements of config #4, profiles/r05_plane_placement.txt)
    const uint64_t need = (ea.row_words / 2 + 255) / 256;
    if (need <= 2) k_emit_wide<256, 2><<<g, 256, 0, st>>>(ea);
    else if (need <= 4) k_emit_wide<256, 4><<<g, 256, 0, st>>>(ea);
    else if (need <= 6) k_emit_wide<256, 6><<<g, 256, 0, st>>>(ea);
    else if (need <= 7) k_emit_wide<256, 7><<<g, 256, 0, st>>>(ea);
    else k_emit_wide<256, 8><<<g, 256, 0, st>>>(ea);
    return need <= 2 ? "k_emit_wide<256,2>" : need <= 4 ? "k_emit_wide<256,4>" : need <= 6 ? "k_emit_wide<256,6>"
         : need <= 7 ? "k_emit_wide<256,7>" : "k_emit_wide<256,8>";
  } else {  // flat multi-row sweep over ~32 KB per block
    ea.chunk = uint32_t(std::min<uint64_t>(EMIT_FLAT_MAX_ROWS, std::max<uint64_t>(1, 32768 / row_bytes)));
    k_emit_flat<256, 8><<<(ea.per_xcd + ea.chunk - 1) / ea.chunk * 8, 256, 0, st>>>(ea);
    return "k_emit_flat<256,8>";
  }
}

static bool enq_emit_blocks(cyc_ctx* c, hipStream_t st, uint64_t* out_in, uint64_t* out_eg, uint8_t* d_status) {
  Problem& pb = c->pb;
  if (pb.blocks.empty()) return false;
  if (!pb.K || !d_status) return true;  // nothing to write (the status plane of blocks is their slabs)
  BlockArgs ba{};
  ba.n_blk = uint32_t(pb.blocks.size());
  ba.K = pb.K;
  ba.AS = c->blk_wa_max;
  ba.blk = c->blk.as<uint4>();
  ba.boff = c->blk_off.as<uint64_t>();
  for (int pl = 0; pl < 2; pl++) {
    ba.pod_id[pl] = c->dir[pl].pod_id.as<uint32_t>();
    ba.class_of[pl] = c->dir[pl].class_of.as<uint32_t>();
    ba.A[pl] = c->dir[pl].A.as<uint64_t>();
  }
  ba.st_src = c->slot_status.as<uint8_t>();
  ba.out[0] = out_in;
  ba.out[1] = out_eg;
  ba.st_out = d_status;
  // a block's slab words split over workgroups of ~16 words per thread (one workgroup per block
  // left a few large blocks on a few CUs); small blocks' extra workgroups exit at once
  const unsigned bs = c->blk_np_max * 2 > 128 ? 256 : 128;
  const uint64_t most = 2ull * c->blk_np_max * pb.K * ((c->blk_np_max + 63) / 64);  // largest slab, both planes
  ba.split = uint32_t(std::min<uint64_t>(64, std::max<uint64_t>(1, most / (uint64_t(bs) * 16))));
  k_emit_blocks<<<ba.n_blk * ba.split, bs, 0, st>>>(ba);
  return true;
}

// part (row phases): 0 = every row of the plan; 1 / 2 = the rows before / from the split (the plan's
// emit lists hold them in that order); the status plane goes with part 1, the span reset with part 2
// (after the last reader of the IP rows' spans, phase 2's class rows).
static bool enq_emit(cyc_ctx* c, hipStream_t st, uint64_t* out_in, uint64_t* out_eg, uint8_t* d_status, bool inplace = false,
                     int part = 0) {
  Problem& pb = c->pb;
  if (part != 1) c->ip_rng_clean = false;  // (set again below when this emit resets the spans for the next run)
  const uint32_t K = pb.K;
  const uint64_t rw[2] = {uint64_t(K) * c->win_wa, uint64_t(K) * pb.W};  // words per plane row
  uint32_t nr[2];
  for (int d = 0; d < 2; d++) nr[d] = rw[d] ? uint32_t(c->rh[d] - c->rl[d]) : 0u;
  if (part != 2) {
    c->emit_kernel.clear();
    c->emit_launches = 0;
  }
  if (!pb.blocks.empty()) {
    const bool r = enq_emit_blocks(c, st, out_in, out_eg, d_status);
    if (r && pb.K && d_status) c->emit_kernel = "k_emit_blocks", c->emit_launches = 1;
    return r;
  }
  if (!nr[0] && !nr[1]) return false;
  EmitArgs ea{};
  ea.st_src = c->slot_status.as<uint8_t>();
  ea.st_dst = d_status;
  ea.st_bytes = d_status ? uint64_t(pb.P) * K : 0;
  ea.reset = c->ip_rng.as<uint32_t>();
  ea.reset_n = pb.may_err ? 0u : uint64_t(pb.peers.size()) * 4;  // (k_ip_rows with panics keeps no spans)
  if (part != 1) c->ip_rng_clean = ea.reset_n != 0;
  for (uint32_t pl = 0; pl < 2; pl++) {
    ea.row_lo[pl] = uint32_t(c->rl[pl]);
    ea.order[pl] = c->order[pl].as<uint2>();
    ea.class_of[pl] = c->dir[pl].class_of.as<uint32_t>();
    ea.A[pl] = c->dir[pl].A.as<uint64_t>();
    ea.arow[pl] = inplace ? c->arow[pl].as<uint32_t>() : nullptr;
  }
  ea.out[0] = out_in;
  ea.out[1] = out_eg;
  ea.pl_words[0] = rw[0];
  ea.pl_words[1] = rw[1];
  auto note = [&](const char* k) {  // what cyc_last_emit reports
    if (c->emit_kernel.find(k) == std::string::npos) c->emit_kernel += (c->emit_kernel.empty() ? "" : " + ") + std::string(k);
    c->emit_launches++;
  };
  if (rw[0] == rw[1] && nr[0] == nr[1]) {  // target rows: both planes in one launch
    ea.row_words = rw[0];
    // alternate the planes' rows when each plane is >= 8 GB (config #3 on one GPU: emit 3.42 ->
    // 3.11 ms on two of three boxes, -1 % on the third; 1-4 % slower for planes of <= 5 GB — 2, 4
    // and 8 shards — profiles/r01_emit_interleave_sweep.txt)
    ea.interleave = c->emit_interleave >= 0 ? uint32_t(c->emit_interleave)
                                            : uint64_t(nr[0]) * rw[0] * 8 >= (8ull << 30) ? 1u : 0u;
    ea.n_rows[0] = ea.n_rows[1] = nr[0];
    if (part) {  // row phases (target rows over the whole table: both planes split at the same row)
      const uint32_t n1 = c->phase_n1[0];
      ea.n_rows[0] = ea.n_rows[1] = part == 1 ? n1 : nr[0] - n1;
      for (int pl = 0; pl < 2; pl++) ea.order[pl] += part == 1 ? 0u : n1;
      if (part == 1) ea.reset_n = 0;
      else ea.st_bytes = 0;
    }
    note(enq_emit_launch(ea, st, out_in, out_eg));
    return true;
  }
  // rows of different lengths (a source shard): ONE launch over units of about one block pass each
  const bool aligned = reinterpret_cast<uintptr_t>(out_in) % 16 == 0 && reinterpret_cast<uintptr_t>(out_eg) % 16 == 0;
  if (aligned && rw[0] % 2 == 0 && rw[1] % 2 == 0) {
    ea.n_rows[0] = nr[0];
    ea.n_rows[1] = nr[1];
    note(enq_emit_units(ea, st));
    return true;
  }
  bool first = true;
  for (int pl = 0; pl < 2; pl++) {  // (8-byte row words or unaligned planes) one launch per plane
    if (!nr[pl]) continue;
    EmitArgs e1 = ea;
    e1.n_rows[0] = pl == 0 ? nr[0] : 0u;  // the row list is [plane 0 rows][plane 1 rows]
    e1.n_rows[1] = pl == 1 ? nr[1] : 0u;
    e1.row_words = rw[pl];
    if (!first) e1.st_bytes = e1.reset_n = 0;
    first = false;
    note(enq_emit_launch(e1, st, pl == 0 ? out_in : reinterpret_cast<uint64_t*>(16), pl == 1 ? out_eg : reinterpret_cast<uint64_t*>(16)));
  }
  return true;
}

// The fused front (k_front_a..e, one stream): the same block ranges the two-branch DAG launches
// as ~15 kernels (enq_common, enq_peer_rows, enq_member, enq_class_rows), grouped by dependency
// level.  Applies to no-panic builds with dense selectors whose pod-peer rows (PM builds) are
// computed per pod in one level; returns false (nothing enqueued) otherwise.
static bool front_fused_ok(const cyc_ctx* c) {
  const Problem& pb = c->pb;
  if (!c->front_fused || pb.may_err) return false;
  if (!pb.P || !pb.K || !pb.W) return false;
  if (uint64_t(c->n_sel) * pb.L && !c->dense_sel) return false;
  if (ido_mode(c)) return true;
  const uint32_t E = c->dir[1].n, Rp = c->rp_off[2] - c->rp_off[0];
  return !(Rp && E) || (c->pod_rows >= 0 ? c->pod_rows == 1 : uint64_t(E) * 2 >= pb.P);
}

// In-place class rows: the fused front with both output planes given.
// Auto (-1): when the rows' identities are >= 1/16 of the rows (PM builds: config #4 emit -8 %,
// #3u -7 %), and for identity-set (IDO) runs: config #3's class rows are 2 % of its rows,
// and writing them into the planes saves their 400 MB of separate writes (3.286 -> 3.191 ms/step,
// profiles/r05_inplace_sweep_ab.txt; over 5 plane placements in one process -2.1 / -0.0 / -0.1 /
// -2.8 / -2.2 %, never slower: profiles/r05_plane_placement.txt; a source shard at N = 8 -1.2 %,
// r05_shard_ab.txt; in round 2, before the current launch E, it lost 1 %).
static bool inplace_ok(const cyc_ctx* c, const uint64_t* d_in, const uint64_t* d_eg) {
  if (!c->class_inplace || !d_in || !d_eg || !front_fused_ok(c) || !c->pb.blocks.empty()) return false;
  const uint64_t rows = uint64_t(std::max<int64_t>((c->rh[0] - c->rl[0] + c->rh[1] - c->rl[1]) / 2, 1));
  return c->class_inplace == 1 || uint64_t(c->n_act[0] + c->n_act[1]) * 16 >= 2 * rows || ido_mode(c);
}

// out_in / out_eg non-null: the class rows go straight into those planes (in-place class rows; the
// emit must then be enqueued with inplace = true).
// mid (row phases, cyc_ctx::phase_split): enqueues phase 1's emit between the two class-row launches;
// ev_mid0 / ev_mid1 (eager runs) bracket phase 2's class rows.
static bool enq_front_fused(cyc_ctx* c, hipStream_t st, hipEvent_t ev_front = nullptr, hipEvent_t ev_rows = nullptr,
                            uint64_t* out_in = nullptr, uint64_t* out_eg = nullptr, const std::function<void()>* mid = nullptr,
                            hipEvent_t ev_mid0 = nullptr, hipEvent_t ev_mid1 = nullptr) {
  Problem& pb = c->pb;
  const uint32_t P = pb.P, K = pb.K, W = pb.W, D = uint32_t(std::max<size_t>(pb.descs.size(), 1));
  const uint32_t M = uint32_t(pb.pms.size()), E = c->dir[1].n, EW = (E + 63) / 64;
  bool fits = true;  // every launch's block count below 2^31 (else the DAG path runs)
  auto blocks = [&fits](uint64_t n) {
    fits = fits && n < (1ull << 30);
    return uint32_t(n);
  };
  // A: IP word spans | port table | slot words | selectors
  FrontA fa{};
  fa.fill_p = c->ip_rng.as<uint32_t>();
  // the word spans and chunk masks of the IP rows and of PM builds' sparse pod rows (cnz needs no reset)
  fa.fill_n = (c->Ri || c->Rr || (!ido_mode(c) && c->Rp)) ? pb.peers.size() * 4 : 0;
  fa.nb[0] = blocks((fa.fill_n + 255) / 256);
  fa.M = M;
  fa.D = D;
  fa.P = P;
  fa.K = K;
  fa.W = W;
  fa.pms = c->pms.as<DPortM>();
  fa.pents = c->pents.as<DPortEntry>();
  fa.descs = c->descs.as<DDesc>();
  fa.portok = c->portok.as<uint8_t>();
  fa.nb[1] = (M && pb.descs.size()) ? blocks((uint64_t(M) * D + 255) / 256) : 0u;
  fa.slot_desc = c->slot_desc.as<int32_t>();
  fa.slot_status = c->slot_status.as<uint8_t>();
  fa.VALID = c->VALID.as<uint64_t>();
  fa.DESCW = c->DESCW.as<int32_t>();
  fa.DM = c->DM.as<uint64_t>();
  // the slot words (VALID / DESCW / DM per 64 destinations) serve only egress class rows whose
  // destinations do not all share each slot's descriptor (uni_desc: the UNI class rows read udesc)
  const bool slot_words = !c->uni_desc || !(ido_mode(c) || pl_wave_ok(c)) || !c->pb.blocks.empty();
  fa.nb[2] = slot_words ? blocks((uint64_t(K) * W + 3) / 4) : 0u;
  fa.S = c->n_sel;
  fa.L = pb.L;
  fa.sel_off = c->sel_off.as<uint32_t>();
  fa.dreqs = c->dreqs.as<DReq>();
  fa.req_vals = c->req_vals.as<uint32_t>();
  fa.LVT = c->lvt.as<uint32_t>();
  fa.selres = c->selres.as<uint8_t>();
  fa.sel_list = c->sel_list.as<uint32_t>();
  fa.nb[3] = uint64_t(c->n_sel) * pb.L && !lazy_sel(c) ? blocks(uint64_t(c->n_sel) * ((pb.L + 256 * SEL_LPT - 1) / (256 * SEL_LPT))) : 0u;
  // B: IP rows | pod-peer identity sets (both directions' adjacent sub-lists) | membership x 2
  // Segments x = 0, 1 of the IP rows and per-pod pod rows: the directions' sub-lists with their own
  // word windows (source shards), or both directions in segment 0 (one window)
  const bool one_win = one_window(c);
  FrontB fb{};
  fb.P = P;
  fb.W = W;
  fb.ip_ex = c->ip_ex.as<DCidr>();
  fb.pod_ip = c->pod_ip.as<DIP>();
  fb.words = c->ip_words.as<DWordIP>();
  fb.PM = c->PM.as<uint64_t>();
  fb.rng = c->ip_rng.as<uint32_t>();
  fb.cnz = ip_cnz(c);
  fb.ip_grp = IP_GROUP;
  fb.ipr_iv = c->ipr_iv.as<uint2>();
  fb.ipsort = c->ipsort.as<uint32_t>();
  fb.ipv_iv = c->ipv_iv.as<uint2>();
  fb.ip_ilist = c->ipi_list.as<uint32_t>();
  for (int x = 0; x < 2; x++) {
    const int dlo = one_win ? 0 : x, dhi = one_win ? 2 : x + 1;
    const uint32_t i0 = c->ri_off[dlo];
    fb.Ri[x] = one_win && x ? 0u : c->ri_off[dhi] - i0;
    fb.tests[x] = c->ip_tests.as<DIPTest>() + i0;
    peer_chunks(c, one_win ? 1 : x, fb.ic0[x], fb.inch[x]);
    fb.nb[x] = fb.Ri[x] && fb.inch[x] ? blocks(ip_rows_blocks(fb.Ri[x], fb.inch[x], fb.ip_grp)) : 0u;
    if (c->ip_items && fb.nb[x]) {  // the range plan's work items of this segment
      fb.ip_items[x] = c->ipi_items.as<DIPItem>() + c->ipi_off[x];
      fb.n_ip_items[x] = c->ipi_off[x + 1] - c->ipi_off[x];
      fb.nb[x] = blocks((uint64_t(fb.n_ip_items[x]) + 3) / 4);
    }
    fb.Rr[x] = one_win && x ? 0u : c->rr_off[dhi] - c->rr_off[dlo];
    fb.rtests[x] = c->ipr_tests.as<DIPRange>() + c->rr_off[dlo];
    fb.nb[9 + x] = fb.Rr[x] && fb.inch[x] ? blocks((uint64_t(fb.Rr[x]) + 3) / 4) : 0u;
    fb.Rv[x] = one_win && x ? 0u : c->rv_off[dhi] - c->rv_off[dlo];
    fb.vtests[x] = c->ipv_tests.as<DIPIv>() + c->rv_off[dlo];
    fb.nb[11 + x] = fb.Rv[x] && fb.inch[x] ? blocks((uint64_t(fb.Rv[x]) + 3) / 4) : 0u;
  }
  fb.E = E;
  fb.EW = EW;
  fb.L = pb.L;
  fb.peers = c->peers.as<DPeer>();
  fb.selres = c->selres.as<uint8_t>();
  fb.id_ns = c->dir[1].id_ns.as<uint32_t>();
  fb.id_nsls = c->id_nsls.as<uint32_t>();
  fb.id_ls = c->dir[1].id_ls.as<uint32_t>();
  fb.sv = sel_view(c);
  fb.word_ns = c->ido_word_ns.as<uint2>();
  for (int x = 0; x < 2; x++) {  // identity sets per direction: the ingress ones over the window's identity words
    const uint32_t ux = c->rpu_off[x];
    fb.Ru_[x] = c->rpu_off[x + 1] - ux;
    fb.pod_peers_u_[x] = c->pod_peers_u.as<uint32_t>() + ux;
    fb.idob_[x] = c->idob.as<uint64_t>() + uint64_t(ux) * EW;
    fb.grp_ns_[x] = c->ido_grp_ns.as<uint2>() + c->ido_goff[x];
    fb.pbrec_[x] = c->pb_rec.p && CYC_PB_REC ? c->pb_rec.as<uint4>() + 3 * uint64_t(ux) : nullptr;
    fb.ew0[x] = x == 0 ? c->ido_ew0 : 0u;
    fb.new_[x] = x == 0 ? c->ido_ew1 - c->ido_ew0 : EW;
    fb.nb[2 + x] = (fb.Ru_[x] && E && fb.new_[x]) ? blocks((uint64_t((fb.Ru_[x] + PB_GROUP - 1) / PB_GROUP) * fb.new_[x] + 3) / 4) : 0u;
  }
  const bool ido = ido_mode(c);
  FrontC fc{};
  if (!ido && !pod_sparse(c)) {  // PM builds, few pod-peer words: full rows, a wave per (pod peer, word)
    fb.pod_direct = 1;
    fb.pod_eid = c->dir[1].pod_id.as<uint32_t>();
    for (int x = 0; x < 2; x++) {
      const int dlo = one_win ? 0 : x, dhi = one_win ? 2 : x + 1;
      fb.Rp[x] = one_win && x ? 0u : c->rp_off[dhi] - c->rp_off[dlo];
      fb.plist[x] = c->pod_peers.as<uint32_t>() + c->rp_off[dlo];
      peer_window(c, one_win ? 1 : x, fb.pw0[x], fb.pnw[x]);
      fb.nb[2 + x] = (fb.Rp[x] && E && fb.pnw[x]) ? blocks((pod_direct_waves(fb.Rp[x], fb.pnw[x]) + 3) / 4) : 0u;
    }
  } else if (!ido) {  // PM builds: sparse pod-peer rows in launch C (k_front_c)
    fb.nb[2] = fb.nb[3] = 0;
    fc.P = P;
    fc.W = W;
    fc.req_post = c->req_post.as<uint4>();
    fc.post_pods = c->post_pods.as<uint32_t>();
    fc.peers = c->peers.as<DPeer>();
    fc.pod_ns = c->pod_ns.as<uint32_t>();
    fc.pod_nsls = c->pod_nsls.as<uint32_t>();
    fc.pod_ls = c->pod_ls.as<uint32_t>();
    fc.nsw = c->ns_words.as<DWordNS>();
    fc.sv = sel_view(c);
    fc.PM = c->PM.as<uint64_t>();
    fc.rng = c->ip_rng.as<uint32_t>();
    fc.cnz = ip_cnz(c);
    // a wave per chunk over groups of 8 peers once that fills the chip (>= 64k peer chunks:
    // config #3u 2.6 vs 3.2 ms), else the 4 waves of a block share each chunk (config #2)
    uint64_t peer_chunks_all = 0;
    for (int x = 0; x < 2; x++) {
      const int dlo = one_win ? 0 : x, dhi = one_win ? 2 : x + 1;
      fc.Rp[x] = one_win && x ? 0u : c->scan_off[dhi] - c->scan_off[dlo];
      fc.plist[x] = c->pp_scan.as<uint32_t>() + c->scan_off[dlo];
      fc.plist_post[x] = c->pp_post.as<uint32_t>() + c->post_off[dlo];
      peer_chunks(c, one_win ? 1 : x, fc.c0[x], fc.nch[x]);
      peer_chunks_all += uint64_t(fc.Rp[x]) * fc.nch[x];
    }
    fc.pr_grp = c->pr_group > 0 ? uint32_t(c->pr_group) : (peer_chunks_all >= 65536 ? 8u : 1u);
    for (int x = 0; x < 2; x++) {
      const int dlo = one_win ? 0 : x, dhi = one_win ? 2 : x + 1;
      const uint64_t cb = (fc.nch[x] + 3) / 4;
      fc.nb[2 + x] = (fc.Rp[x] && E && cb) ? blocks((uint64_t(fc.Rp[x]) + fc.pr_grp - 1) / fc.pr_grp * cb) : 0u;
      fc.nb[4 + x] = E && fc.nch[x] && !(one_win && x) ? c->post_off[dhi] - c->post_off[dlo] : 0u;  // a block per posting-built peer
    }
  }
  FrontRows fd{}, fe{};
  size_t lds = 0, lds_uni = 0, e_per[2] = {0, 0};
  uint32_t e_na[2] = {0, 0};
  // row phases: the class rows in two launches with phase 1's emit between them (the caller's mid)
  const bool phases = c->phase_split && mid;
  c->phase_used = phases ? 2 : 0;
  for (int d = 0; d < 2; d++) {
    const uint32_t na = c->dir[d].n ? c->n_act[d] : 0u;
    fb.ma[d] = member_args(c, d);
    fc.ma[d] = fb.ma[d];
    if (phases) {  // the class election lists phase 2's classes apart (from the tail of reps[])
      fc.ma[d].first_row = c->arow[d].as<uint32_t>();
      fc.ma[d].split = c->phase_split;
    }
    fc.class_of[d] = c->dir[d].class_of.as<uint32_t>();
    fb.member_wave[d] = c->member_wave > 0 || (c->member_wave < 0 && na <= 4096 && c->act_targets[d] >= 4.0);
    fb.nb[4 + d] = na ? blocks(fb.member_wave[d] ? (uint64_t(na) + 3) / 4 : (uint64_t(na) + 255) / 256) : 0u;
    fc.nb[d] = na ? blocks((uint64_t(na) + 255) / 256) : 0u;
    if (!na) continue;
    fd.ra[d] = row_args(c, d);  // its blocks empty the direction's hash table for the next run
    if (out_in && out_eg) {
      fd.ra[d].A = d == 0 ? out_in : out_eg;
      fd.ra[d].arow = c->arow[d].as<uint32_t>();
    }
    // (the class election keeps a launch of its own, C: electing inside the next launch's blocks put
    // the election chain on every block — IDO identity sets C + D 29 -> 45 us, PM class rows C + D
    // 79 -> 117 us on config #4: profiles/r04_elect_ab.txt)
    if (!ido) {  // PM builds: launch D (k_front_d_pm) is the class rows from flattened peer lists
      fd.nb[d] = pl_blocks(c, d);
      if (d == 1 && c->uni_desc && c->pb.blocks.empty()) fd.ra[d].udesc = c->udesc.as<int32_t>();
      fd.ra[d].pod_sparse = pod_sparse(c);  // pod rows from pod_rows_sparse_blk (launch C)
      continue;
    }
    fe.ra[d] = fd.ra[d];
    fe.ra[d].ht_clear_words = 0;  // (launch D's identity sets empty it)
    fd.nb[d] = blocks((uint64_t(na) * ((fd.ra[d].NB + CI_G - 1) / CI_G) + 3) / 4);
    // egress with one descriptor per slot (udesc): only the block's slots' sets are staged
    if (d == 1 && c->uni_desc) fe.ra[d].udesc = c->udesc.as<int32_t>();
    e_per[d] = size_t(d == 0 || fe.ra[d].udesc ? uint32_t(E_KC) : D) * fd.ra[d].EW * 8 +
               IDO_IPL * sizeof(uint4) + 16;  // identity sets + staged IP peers (+ alignment)
    e_na[d] = na;
  }
  // launch E's representatives per block: the most of 16 / 8 that still leaves >= 3000 blocks
  // (about two rounds of the chip's resident blocks: one block's staging latency is paid once per
  // 16 representatives), else 4 (config #3: E 106 -> 96 us at N = 1 with 16; at N = 8 a source
  // shard's ~1,900 blocks of 4 ran 22.8 us, of 8 24.0 — profiles/r04_class_rpb_ab.txt).  With row
  // phases each of the two launches computes about half of the classes, so half of its blocks count
  // (config #3 phased E per step, 8 per block against 16: 121.4 vs 141.8 us on one box, 122.8 vs 123.8
  // on another — profiles/r06_class_rpb_ab.txt)
  auto e_blocks = [&](int d, uint32_t rpb) {
    return uint64_t(ido_chunk_groups(fe.ra[d].WA)) * ((K + E_KC - 1) / E_KC) * ((e_na[d] + rpb - 1) / rpb);
  };
  uint32_t e_want = uint32_t(c->class_rpb_opt);
  if (!e_want) {
    e_want = 4;
    for (uint32_t cand : {16u, 8u}) {
      uint64_t tot = 0;
      for (int d = 0; d < 2; d++)
        if (e_per[d]) tot += e_blocks(d, class_rpb(c, e_per[d], cand));
      if ((phases ? tot / 2 : tot) >= 3000) {
        e_want = cand;
        break;
      }
    }
  }
  for (int d = 0; d < 2; d++) {
    if (!e_per[d]) continue;
    fe.ra[d].rpb = class_rpb(c, e_per[d], e_want);
    fe.nb[d] = blocks(e_blocks(d, fe.ra[d].rpb));
    if (d == 1 && fe.ra[d].udesc) lds_uni = e_per[d] * fe.ra[d].rpb;
    else lds = std::max<size_t>(lds, e_per[d] * fe.ra[d].rpb);
  }
  // membership ahead of the rest of launch B unless the IP rows alone fill the chip (~2k resident blocks)
  fb.member_first = uint64_t(fb.nb[0]) + fb.nb[1] < 2048;
  const bool bits = fa.nb[1] && port_bits_on(c);
  const uint32_t nb_bits = bits ? blocks((uint64_t(M) + 255) / 256) : 0u;
  fb.M = M;
  fb.D = D;
  fb.portok = c->portok.as<uint8_t>();
  fb.portbits = c->portbits.as<uint32_t>();
  fb.nb[6] = nb_bits;
  fe.ra[1].portbits = bits && fe.nb[1] ? c->portbits.as<uint32_t>() : nullptr;
  // Without a selector table to build (lazy selectors) launch A is dropped: its port table, slot
  // words and port bits (from the matchers directly) join launch B — their readers are the class
  // rows, launches D / E — and the IP rows' word spans were reset by the previous run's emit
  // (EmitArgs::reset; a memset when they were not).  Captured graphs keep launch A: a replay must not
  // depend on the step before it.
  if (fa.nb[3] == 0 && !c->capturing) {
    fb.pre = fa;
    fb.bits_direct = 1;
    fb.nb[7] = fa.nb[1];
    fb.nb[8] = fa.nb[2];
    if (fa.fill_n && !c->ip_rng_clean) HIPCHK(hipMemsetAsync(fa.fill_p, 0xFF, fa.fill_n * 4, st));
    fa.nb[0] = fa.nb[1] = fa.nb[2] = 0;
  }
  const uint64_t ga = uint64_t(fa.nb[0]) + fa.nb[1] + fa.nb[2] + fa.nb[3];
  uint64_t gb = 0, gc = 0;
  for (uint32_t x : fb.nb) gb += x;
  for (uint32_t x : fc.nb) gc += x;
  if (!fits || gb >= (1ull << 31) || gc >= (1ull << 31)) return false;
  if (ga) k_front_a<<<unsigned(ga), 256, 0, st>>>(fa);
  if (gb) k_front_b<<<unsigned(gb), 256, 0, st>>>(fb);
  if (gc) k_front_c<<<unsigned(gc), 256, 0, st>>>(fc);
  if (ev_front) HIPCHK(hipEventRecord(ev_front, st));  // eager runs: phase timings
  // the class rows: once, or per row phase with phase 1's emit between (the caller's mid)
  // a phased launch's grid covers only the identities that can represent its phase's classes (the
  // representatives' first rows decide the phase), not every active identity
  const uint32_t fd_all[2] = {fd.nb[0], fd.nb[1]}, fe_all[2] = {fe.nb[0], fe.nb[1]};
  auto class_rows = [&](uint32_t phase) {
    for (int d = 0; d < 2; d++) {
      RowArgs& ra = ido ? fe.ra[d] : fd.ra[d];
      ra.phase = phase;
      if (!CYC_PHASE_GRID || !phase) continue;
      const uint32_t na = c->dir[d].n ? c->n_act[d] : 0u;
      const uint32_t nph = phase == 1 ? c->n_act_ph1[d] : na - c->n_act_ph1[d];
      if (ido) {
        if (fe_all[d]) fe.nb[d] = blocks(uint64_t(ido_chunk_groups(fe.ra[d].WA)) * ((K + E_KC - 1) / E_KC) *
                                         ((nph + fe.ra[d].rpb - 1) / fe.ra[d].rpb));
      } else if (fd_all[d]) {
        fd.nb[d] = std::min(fd_all[d], nph);
      }
    }
    if (!ido) {
      const unsigned gd = fd.nb[0] + fd.nb[1];
      if (gd && pl_wave_ok(c)) k_front_d_pm<true><<<gd, pl_threads(c), 0, st>>>(fd);
      else if (gd) k_front_d_pm<false><<<gd, pl_threads(c), 0, st>>>(fd);
    } else if (fe.nb[0] && fe.nb[1] && fe.ra[1].udesc) {
      k_front_e_uni<<<fe.nb[0] + fe.nb[1], 256, std::max(lds, lds_uni), st>>>(fe);
    } else {  // the directions' class rows as two launches, each at its own register budget (egress 101
              // VGPRs, ingress 61: one launch at 101 ran config #3 189 -> 170 us, profiles/r03_e_split_ab.txt)
      if (fe.nb[1] && fe.ra[1].udesc) k_class_rows_ido<true, E_KC, true><<<fe.nb[1], 256, lds_uni, st>>>(fe.ra[1]);
      else if (fe.nb[1]) k_class_rows_ido<true, E_KC><<<fe.nb[1], 256, lds, st>>>(fe.ra[1]);
      if (fe.nb[0]) k_class_rows_ido<false, E_KC><<<fe.nb[0], 256, lds, st>>>(fe.ra[0]);
    }
  };
  if (ido && fd.nb[0] + fd.nb[1]) k_front_d<<<fd.nb[0] + fd.nb[1], 256, 0, st>>>(fd);  // identity sets: once
  class_rows(phases ? 1u : 0u);
  if (ev_rows) HIPCHK(hipEventRecord(ev_rows, st));
  if (phases) {
    (*mid)();
    if (ev_mid0) HIPCHK(hipEventRecord(ev_mid0, st));
    class_rows(2u);
    if (ev_mid1) HIPCHK(hipEventRecord(ev_mid1, st));
  }
  return true;
}

// Eager launch, in phase order with the timing events: [0] start, [1] after the front (peer
// rows, classes), [2] after the class rows, [3] after both emits.
static void enqueue_pipeline(cyc_ctx* c, hipStream_t st, uint64_t* d_in, uint64_t* d_eg, uint8_t* d_status) {
  Problem& pb = c->pb;
  HIPCHK(hipEventRecord(c->ev[0], st));
  const bool ip = inplace_ok(c, d_in, d_eg);
  c->phase_used = 0;
  const std::function<void()> mid = [&] { enq_emit(c, st, d_in, d_eg, d_status, ip, 1); };
  const bool fused = front_fused_ok(c) && enq_front_fused(c, st, c->ev[1], c->ev[2], ip ? d_in : nullptr, ip ? d_eg : nullptr,
                                                          &mid, c->ev_p[0], c->ev_p[1]);
  if (!fused) {
    enq_common(c, st);
    for (int d = 0; d < 2; d++) enq_peer_rows(c, d, st);
    for (int d = 0; d < 2; d++) enq_member(c, d, st);
    HIPCHK(hipEventRecord(c->ev[1], st));
    for (int d = 0; d < 2; d++) enq_class_rows(c, d, st);
    HIPCHK(hipEventRecord(c->ev[2], st));
  }
  const bool status_done = enq_emit(c, st, d_in, d_eg, d_status, ip && fused, c->phase_used ? 2 : 0);
  HIPCHK(hipEventRecord(c->ev[3], st));
  if (!status_done && d_status && uint64_t(pb.P) * pb.K)
    HIPCHK(hipMemcpyAsync(d_status, c->slot_status.p, uint64_t(pb.P) * pb.K, hipMemcpyDeviceToDevice, st));
}

// Graph capture / eager DAG: the fused front on st when it applies; else the two-branch DAG:
// [st3] IP rows of both directions + port tables || [st] selectors, then per direction (ingress on
// st, egress on st2) pod-peer sets -> membership / classes -> (wait for st3) class rows, joined
// into one emit of both planes (fork / join through events, graph dependencies when captured).
static void capture_pipeline(cyc_ctx* c, hipStream_t st, hipStream_t st2, hipStream_t st3, uint64_t* d_in, uint64_t* d_eg,
                             uint8_t* d_status) {
  Problem& pb = c->pb;
  const bool ip = inplace_ok(c, d_in, d_eg);
  c->phase_used = 0;
  const std::function<void()> mid = [&] { enq_emit(c, st, d_in, d_eg, d_status, ip, 1); };
  if (front_fused_ok(c) && enq_front_fused(c, st, nullptr, nullptr, ip ? d_in : nullptr, ip ? d_eg : nullptr, &mid)) {
    if (enq_emit(c, st, d_in, d_eg, d_status, ip, c->phase_used ? 2 : 0)) return;
  } else {
    HIPCHK(hipEventRecord(c->fork_ev, st));
    HIPCHK(hipStreamWaitEvent(st3, c->fork_ev, 0));
    enq_common(c, st3, COMMON_FILL | COMMON_PORTS);
    enq_peer_rows(c, 2, st3, PEERS_IP);  // both directions' IP rows in one launch
    HIPCHK(hipEventRecord(c->ports_ev, st3));
    enq_common(c, st, COMMON_SELECTORS);
    HIPCHK(hipEventRecord(c->sel_ev, st));
    HIPCHK(hipStreamWaitEvent(st2, c->sel_ev, 0));
    for (int d = 1; d >= 0; d--) {
      hipStream_t s = d ? st2 : st;
      enq_peer_rows(c, d, s, PEERS_POD);
      enq_member(c, d, s);
      HIPCHK(hipStreamWaitEvent(s, c->ports_ev, 0));
      enq_class_rows(c, d, s);
    }
    HIPCHK(hipEventRecord(c->join_ev, st2));
    HIPCHK(hipStreamWaitEvent(st, c->join_ev, 0));
    // the emit also writes the status plane; the copy node below only ends steps without rows
    if (enq_emit(c, st, d_in, d_eg, d_status)) return;
  }
  // The step always ends with the status-plane copy (into a sink buffer when the caller passed no
  // status pointer), so every captured graph has the same shape: one node after the join.
  const uint64_t nst = uint64_t(pb.P) * pb.K;
  uint8_t* dst = d_status && nst ? d_status : c->status_sink.as<uint8_t>();  // sink: >= 16 B (prepare_device)
  HIPCHK(hipMemcpyAsync(dst, c->slot_status.p, std::max<uint64_t>(nst, 1), hipMemcpyDeviceToDevice, st));
}

// Destroy the retired execs whose last launch has completed (all of them when `wait`).
static void reap_graphs(cyc_ctx* c, bool wait) {
  size_t keep = 0;
  for (size_t i = 0; i < c->retired.size(); i++) {
    cyc_ctx::Retired& r = c->retired[i];
    if (r.done && wait) (void)hipEventSynchronize(r.done);
    const bool done = !r.done || wait || hipEventQuery(r.done) != hipErrorNotReady;
    if (!done) {
      c->retired[keep++] = r;
      continue;
    }
    (void)hipGraphExecDestroy(r.exec);
    if (r.graph) (void)hipGraphDestroy(r.graph);
    if (r.done) (void)hipEventDestroy(r.done);
  }
  c->retired.resize(keep);
}

static void drop_graph(cyc_ctx* c) {
  if (c->graph_exec) c->retired.push_back({c->graph_exec, c->graph, c->graph_done});
  c->graph_exec = nullptr;
  c->graph = nullptr;
  c->graph_done = nullptr;
  reap_graphs(c, false);
}

static void ensure_cap_streams(cyc_ctx* c) {
  if (c->cap_stream) return;
  HIPCHK(hipStreamCreateWithFlags(&c->cap_stream, hipStreamNonBlocking));
  HIPCHK(hipStreamCreateWithFlags(&c->cap_stream2, hipStreamNonBlocking));
  HIPCHK(hipStreamCreateWithFlags(&c->cap_stream3, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&c->sel_ev, EV_SYNC));
  HIPCHK(hipEventCreateWithFlags(&c->ports_ev, EV_SYNC));
  HIPCHK(hipEventCreateWithFlags(&c->fork_ev, EV_SYNC));
  HIPCHK(hipEventCreateWithFlags(&c->join_ev, EV_SYNC));
}

// Batched blocks: each block's status, as its stand-alone run would end — the job expansion's
// panic, else its first panicking job (its own job order), else its table build's duplicate key —
// into c->blk_rc / c->blk_msg.  Synchronises only when the inputs can panic.
static int blocks_status(cyc_ctx* c, hipStream_t st) {
  Problem& pb = c->pb;
  const size_t nb = pb.blocks.size();
  c->blk_rc.assign(nb, CYC_OK);
  c->blk_msg.assign(nb, "");
  std::vector<unsigned long long> first(nb, ~0ull);
  if (pb.may_err && pb.P && pb.K) {
    HIPCHK(hipMemsetAsync(c->first_blk.p, 0xFF, nb * 8, st));
    BlockErrArgs e{};
    e.n_blk = uint32_t(nb);
    e.P = pb.P;
    e.K = pb.K;
    e.AS = c->blk_wa_max;
    e.blk = c->blk.as<uint4>();
    e.pod_blk = nullptr;
    e.slot_idx = c->slot_idx.as<uint32_t>();
    e.slot_status = c->slot_status.as<uint8_t>();
    e.pod_iid = c->dir[0].pod_id.as<uint32_t>();
    e.pod_eid = c->dir[1].pod_id.as<uint32_t>();
    e.class_in = c->dir[0].class_of.as<uint32_t>();
    e.class_eg = c->dir[1].class_of.as<uint32_t>();
    e.err_in = c->dir[0].err.as<uint8_t>();
    e.err_eg = c->dir[1].err.as<uint8_t>();
    e.AE_in = c->dir[0].AE.as<uint64_t>();
    e.AE_eg = c->dir[1].AE.as<uint64_t>();
    e.first = c->first_blk.as<unsigned long long>();
    e.dchunks = (c->blk_np_max + 255) / 256;
    DevBuf pod_blk;
    upload(pod_blk, pb.pod_blk);
    e.pod_blk = pod_blk.as<uint32_t>();
    if (c->dir[0].n && c->dir[1].n)
      k_first_error_blocks<<<grid1(uint64_t(pb.P) * e.dchunks, 1), 256, 0, st>>>(e);
    HIPCHK(hipMemcpyAsync(first.data(), c->first_blk.p, nb * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  const std::string saved = c->err;
  for (size_t b = 0; b < nb; b++) {
    const ProbeBlock& x = pb.blocks[b];
    if (pb.blk_expand_panic[b]) {
      c->blk_rc[b] = CYC_ERR_PANIC_RUNTIME;
      c->blk_msg[b] = "runtime error: index out of range [0] with length 0";
    } else if (first[b] != ~0ull) {
      const uint32_t np = x.p1 - x.p0, idx = uint32_t(first[b] % 65536);
      const uint64_t rest = first[b] / 65536;
      c->blk_rc[b] = describe_panic(c, x.p0 + uint32_t(rest / np), x.p0 + uint32_t(rest % np), x.cfg, idx);
      c->blk_msg[b] = c->err;
    } else if (!pb.blk_dup_msg[b].empty()) {
      c->blk_rc[b] = CYC_ERR_DUPLICATE_KEY;
      c->blk_msg[b] = pb.blk_dup_msg[b];
    }
  }
  c->err = saved;
  return (int)CYC_OK;
}

// allow_capture = false: never capture a graph for this run (cyc_table_run's planes are new on
// every call, so a captured graph would be re-instantiated each time): graphs = 1 runs as 2.
// src: rows [lo, hi) are a source shard (CYC_ROWS_SOURCE), else target rows.
static int run_pipeline(cyc_ctx* c, hipStream_t st, uint64_t* d_in, uint64_t* d_eg, uint8_t* d_status, int64_t lo,
                        int64_t hi, bool allow_capture = true, bool src = false) {
  Problem& pb = c->pb;
  const uint32_t P = pb.P, K = pb.K, W = pb.W;
  if (lo < 0 || hi > int64_t(P) || lo > hi) return fail(c, CYC_ERR_ARG, "row range out of bounds");
  if (src && (lo % 64 || (hi % 64 && hi != int64_t(P))))
    return fail(c, CYC_ERR_ARG, "source rows: row_lo must be a multiple of 64, row_hi too unless it is the pod count");
  if (c->order_lo != lo || c->order_hi != hi || c->order_src != src) drop_graph(c);  // range plan buffers are re-made
  ensure_range(c, lo, hi, src);
  if (!c->plvt_ready && front_fused_ok(c) && pod_sparse(c)) {
    drop_graph(c);  // a graph captured without the per-pod table would keep the slower gathers
    ensure_plvt(c, st);
  }
  int graphs = c->use_graphs >= 0 ? c->use_graphs : (front_fused_ok(c) ? 2 : 1);
  if (graphs == 1 && !allow_capture) graphs = 2;
  if (graphs == 2 && !pb.may_err) {
    // the graph's DAG, enqueued directly: the caller's stream forks to two internal streams and
    // joins them back before the emit (events), without hipGraphLaunch's per-replay latency
    ensure_cap_streams(c);
    if (c->step_events) HIPCHK(hipEventRecord(c->ev[0], st));
    capture_pipeline(c, st, c->cap_stream2, c->cap_stream3, d_in, d_eg, d_status);
    if (c->step_events) HIPCHK(hipEventRecord(c->ev[3], st));
    c->timed = c->step_events != 0;
    c->timed_graph = true;
  } else if (graphs && !pb.may_err) {
    // The whole pipeline as one hipGraph (captured once per output buffers / row range):
    // removes the host launch cost of ~16 launches per run (dominant on small problems).
    const void* key[6] = {d_in, d_eg, d_status, reinterpret_cast<void*>(lo), reinterpret_cast<void*>(hi),
                          reinterpret_cast<void*>(intptr_t(src))};
    if (!c->graph_exec || memcmp(key, c->graph_key, sizeof(key)) != 0) {
      drop_graph(c);
      ensure_cap_streams(c);
      hipGraph_t g = nullptr;
      HIPCHK(hipStreamBeginCapture(c->cap_stream, hipStreamCaptureModeThreadLocal));
      c->capturing = true;
      try {
        capture_pipeline(c, c->cap_stream, c->cap_stream2, c->cap_stream3, d_in, d_eg, d_status);
      } catch (...) {
        c->capturing = false;
        throw;
      }
      c->capturing = false;
      HIPCHK(hipStreamEndCapture(c->cap_stream, &g));
      c->graph = g;  // destroyed with the exec (drop_graph / reap_graphs)
      HIPCHK(hipGraphInstantiate(&c->graph_exec, g, nullptr, nullptr, 0));
      HIPCHK(hipEventCreateWithFlags(&c->graph_done, EV_SYNC));
      memcpy(c->graph_key, key, sizeof(key));
    }
    if (c->step_events) HIPCHK(hipEventRecord(c->ev[0], st));
    HIPCHK(hipGraphLaunch(c->graph_exec, st));
    HIPCHK(hipEventRecord(c->graph_done, st));  // the exec may be retired once this completes
    if (c->step_events) HIPCHK(hipEventRecord(c->ev[3], st));
    c->timed = c->step_events != 0;
    c->timed_graph = true;
  } else {
    enqueue_pipeline(c, st, d_in, d_eg, d_status);
    c->timed = true;
    c->timed_graph = false;
  }
  c->ran = true;
  c->last_stream = st;  // cyc_last_classes waits for this stream only

  if (!pb.blocks.empty()) return blocks_status(c, st);

  // 8. panic path: the first panicking job in job order, as the reference would hit it.  Configs
  // run in order (one RunProbeForConfig each); within one, the job expansion (may panic on a pod
  // without containers) precedes the evaluation, which precedes the table build (duplicate keys).
  uint32_t eval_cfg = pb.n_cfg, eval_s = 0, eval_d = 0, eval_idx = 0;
  if (pb.may_err) {
    if (P >= (1u << 24) || K > 65536)  // k_first_error's job-order key: (s*P + d)*65536 + idx < 2^64
      throw Panic{CYC_ERR_ARG, "inputs that can panic are limited to 2^24 pods and 65536 job slots"};
    HIPCHK(hipMemsetAsync(c->first_err.p, 0xFF, uint64_t(pb.n_cfg) * 8, st));
    ErrArgs e{};
    e.P = P;
    e.K = K;
    e.W = W;
    e.n_cfg = pb.n_cfg;
    e.row_lo = uint32_t(lo);
    e.row_hi = uint32_t(hi);
    e.src = src ? 1u : 0u;
    e.w0 = c->win_w0;
    e.WA = c->win_wa;
    e.slot_status = c->slot_status.as<uint8_t>();
    e.slot_cfg = c->slot_cfg.as<uint32_t>();
    e.slot_idx = c->slot_idx.as<uint32_t>();
    e.pod_iid = c->dir[0].pod_id.as<uint32_t>();
    e.pod_eid = c->dir[1].pod_id.as<uint32_t>();
    e.class_in = c->dir[0].class_of.as<uint32_t>();
    e.class_eg = c->dir[1].class_of.as<uint32_t>();
    e.err_in = c->dir[0].err.as<uint8_t>();
    e.err_eg = c->dir[1].err.as<uint8_t>();
    e.AE_in = c->dir[0].n ? c->dir[0].AE.as<uint64_t>() : nullptr;
    e.AE_eg = c->dir[1].n ? c->dir[1].AE.as<uint64_t>() : nullptr;
    e.first = c->first_err.as<unsigned long long>();
    if (P && K) k_first_error<<<grid1(uint64_t((P + 255) / 256) * P, 1), 256, 0, st>>>(e);
    std::vector<unsigned long long> first(std::max<uint32_t>(pb.n_cfg, 1), ~0ull);
    HIPCHK(hipMemcpyAsync(first.data(), c->first_err.p, uint64_t(pb.n_cfg) * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    for (uint32_t cc = 0; cc < pb.n_cfg; cc++)
      if (first[cc] != ~0ull) {
        eval_cfg = cc;
        eval_idx = uint32_t(first[cc] % 65536);
        const uint64_t rest = first[cc] / 65536;
        eval_d = uint32_t(rest % P);
        eval_s = uint32_t(rest / P);
        break;
      }
  }
  for (uint32_t cc = 0; cc < pb.n_cfg; cc++) {
    if (pb.expand_panic[cc]) return fail(c, CYC_ERR_PANIC_RUNTIME, "runtime error: index out of range [0] with length 0");
    if (cc == eval_cfg) return describe_panic(c, eval_s, eval_d, eval_cfg, eval_idx);
    if (!pb.dup_key_msg[cc].empty()) return fail(c, CYC_ERR_DUPLICATE_KEY, pb.dup_key_msg[cc]);
  }
  return (int)CYC_OK;
}

// Host-side formatting of the panic message for the identified first panicking job.  The
// device found WHICH job panics; this re-derives the reference's message text for it by
// replaying that single job's evaluation order over the compiled tables (error path only).
int describe_panic(cyc_ctx* c, uint32_t s, uint32_t d, uint32_t cfg, uint32_t idx) {
  Problem& pb = c->pb;
  uint32_t k = 0;
  for (uint32_t kk = 0; kk < pb.K; kk++)
    if (pb.slot_cfg[kk] == cfg && pb.slot_idx[kk] == idx) k = kk;
  std::vector<uint8_t> selres(size_t(pb.S) * pb.L);
  HIPCHK(hipMemcpy(selres.data(), c->selres.p, selres.size(), hipMemcpyDeviceToHost));
  auto sel = [&](uint32_t sid, uint32_t ls) { return selres[size_t(sid) * pb.L + ls]; };
  auto ip_err = [&](const DPeer& pr, uint32_t q, std::string& msg) -> int {
    const DIPBlock& b = pb.ipbs[pr.ipb];
    auto cidr_msg = [&](uint32_t id) {
      return "unable to parse CIDR '" + pb.cidr_str[id] + "': invalid CIDR address: " + pb.cidr_str[id];
    };
    if (!pb.cidrs[b.cidr].valid) {
      msg = cidr_msg(b.cidr);
      return CYC_ERR_PANIC_CIDR;
    }
    if (!pb.pod_ip[q].valid) {
      msg = "unable to parse IP '" + pb.pod_ip_str[q] + "'";
      return CYC_ERR_PANIC_IP;
    }
    for (uint32_t e = 0; e < b.excnt; e++) {
      uint32_t x = pb.ipb_ex[b.exoff + e];
      if (!pb.cidrs[x].valid) {
        msg = cidr_msg(x);
        return CYC_ERR_PANIC_CIDR;
      }
    }
    return 0;
  };
  // direction 0 (ingress): target d, peer s; direction 1 (egress): target s, peer d
  for (int dir = 0; dir < 2; dir++) {
    uint32_t tp = dir == 0 ? d : s, peer = dir == 0 ? s : d;
    uint32_t ns = pb.pod_ns[tp], ls = pb.pod_ls[tp];
    uint32_t lo = pb.tns_lo[dir][ns], hi = pb.tns_hi[dir][ns];
    for (uint32_t t = lo; t < hi; t++)
      if (sel(pb.tgt[dir][t].sel, ls) == 2) return fail(c, CYC_ERR_PANIC_SELECTOR, "invalid operator");
    // copy of the device outcome rows for the peer pod's word
    for (uint32_t t = lo; t < hi; t++) {
      if (sel(pb.tgt[dir][t].sel, ls) != 1) continue;
      const DTarget& tg = pb.tgt[dir][t];
      for (uint32_t j = tg.poff; j < tg.poff + tg.pcnt; j++) {
        const DPeer& pr = pb.peers[j];
        if (pr.kind == 0) break;
        int32_t de = pb.slot_desc[size_t(d) * pb.K + k];
        std::vector<uint8_t> ok(1);
        HIPCHK(hipMemcpy(ok.data(), c->portok.as<uint8_t>() + size_t(pr.port) * std::max<size_t>(pb.descs.size(), 1) + de, 1,
                         hipMemcpyDeviceToHost));
        if (pr.kind == 1) {
          if (ok[0]) break;
          continue;
        }
        uint64_t pm, er;
        const size_t row = pr.kind == 3 && j < c->prow_host.size() ? c->prow_host[j] : j;  // IP peers share their IPBlock's row
        HIPCHK(hipMemcpy(&pm, c->PM.as<uint64_t>() + row * pb.W + peer / 64, 8, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(&er, c->ER.as<uint64_t>() + row * pb.W + peer / 64, 8, hipMemcpyDeviceToHost));
        if ((er >> (peer % 64)) & 1) {
          if (pr.kind == 2) return fail(c, CYC_ERR_PANIC_SELECTOR, "invalid operator");
          std::string msg;
          int code = ip_err(pr, peer, msg);
          return fail(c, code ? code : CYC_ERR_PANIC_CIDR, msg);
        }
        if (((pm >> (peer % 64)) & 1) && ok[0]) break;
      }
    }
  }
  return fail(c, CYC_ERR_PANIC_CIDR, "panic (unresolved message)");
}

static void destroy_events(cyc_ctx* c) {
  for (auto& e : c->ev)
    if (e) {
      (void)hipEventDestroy(e);
      e = nullptr;
    }
  for (auto& e : c->ev_p)
    if (e) {
      (void)hipEventDestroy(e);
      e = nullptr;
    }
}
