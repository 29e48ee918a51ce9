// lz4e_window2.h -- the greedy parse in windows of 128 positions, two per
// lane.  Part of lz4e_compress.hip's translation unit: included inside its
// anonymous namespace after compress_block, whose helpers it uses.
//
// The algorithm is compress_block's (the reference greedy parse,
// /root/reference/lz4e/lz4e_compress.c:218-534, restated there position by
// position); only the window changes.  Lane l holds positions B + l (half 0)
// and B + 64 + l (half 1), so the chain of dependent cross-lane steps a
// window pays once -- table snapshot, speculative put and read-back, the
// clash ballots, the chain-table compositions, the serial walk's exits, the
// emit's scan, the commit -- covers ~130 input bytes instead of ~65.
//  * masks over the window are pairs of u64 (M2, bit x = position B + x);
//  * per-position fields of <= 16 bits (next chain position, last probe)
//    travel packed, half 1 in the high 16 bits, so a gather at a per-lane
//    position is one ds_bpermute and a walk step one v_readlane per table;
//  * a clash lane's candidate (an earlier window position) is matched
//    against bytes re-read from L1 instead of gathered from the other lane's
//    registers (which half holds them is per lane).
// Dictionary mode stays with compress_block.

struct M2 {
    uint64_t lo, hi;
};
LZ4E_DEV M2 operator|(M2 a, M2 b) { return {a.lo | b.lo, a.hi | b.hi}; }
LZ4E_DEV M2 operator&(M2 a, M2 b) { return {a.lo & b.lo, a.hi & b.hi}; }
LZ4E_DEV M2 operator^(M2 a, M2 b) { return {a.lo ^ b.lo, a.hi ^ b.hi}; }
LZ4E_DEV M2 operator~(M2 a) { return {~a.lo, ~a.hi}; }
LZ4E_DEV bool m2_any(M2 a) { return (a.lo | a.hi) != 0; }
LZ4E_DEV M2 m2_bit(uint32_t x) {
    const uint64_t b = 1ull << (x & 63);
    return {x < 64 ? b : 0, x < 64 ? 0 : b};
}
// positions < x (x <= 128)
LZ4E_DEV M2 m2_below(uint32_t x) {
    if (x >= 128) return {~0ull, ~0ull};
    if (x >= 64) return {~0ull, (1ull << (x - 64)) - 1};
    return {(1ull << x) - 1, 0};
}
// positions a..b (a <= b <= 127)
LZ4E_DEV M2 m2_range(uint32_t a, uint32_t b) { return m2_below(b + 1) & ~m2_below(a); }
// lowest position, 128 if none
LZ4E_DEV uint32_t m2_ctz(M2 a) { return a.lo ? ctz64(a.lo) : (a.hi ? 64 + ctz64(a.hi) : 128); }
// highest position, -1 if none
LZ4E_DEV int32_t m2_top(M2 a) {
    return a.hi ? 127 - (int32_t)__builtin_clzll(a.hi)
                : (a.lo ? 63 - (int32_t)__builtin_clzll(a.lo) : -1);
}
LZ4E_DEV uint32_t m2_popc(M2 a) { return popc64(a.lo) + popc64(a.hi); }
LZ4E_DEV M2 m2_shr2(M2 a) { return {(a.lo >> 2) | (a.hi << 62), a.hi >> 2}; }
LZ4E_DEV M2 ballot2(bool p0, bool p1) { return {ballot(p0), ballot(p1)}; }
// bit of my half-h position (h compile-time)
LZ4E_DEV bool half_bit(M2 a, uint32_t h, uint32_t lane) { return ((h ? a.hi : a.lo) >> lane) & 1; }
// positions below my half-h position
LZ4E_DEV M2 below_me(uint32_t h, uint64_t lanes_below) {
    return h ? M2{~0ull, lanes_below} : M2{lanes_below, 0};
}
// window position x's value (x wave-uniform) of a per-half pair
LZ4E_DEV uint32_t pos_val(const uint32_t* v, uint32_t x) {
    const uint32_t l = x & 63;
    return x < 64 ? lane_val(v[0], l) : lane_val(v[1], l);
}
// Packed per-position fields: position x's (x wave-uniform) and, per lane,
// the field of position idx < 128 (one ds_bpermute).
LZ4E_DEV uint32_t pk2(uint32_t f0, uint32_t f1) { return f0 | (f1 << 16); }
LZ4E_DEV uint32_t pk_shfl(uint32_t pk, uint32_t idx) {
    return (shfl(pk, idx) >> ((idx >> 2) & 16)) & 0xFFFFu;
}

template <int TT, bool kStamps, class IMG>
LZ4E_DEV void compress_block_w2(const IMG& img, uint32_t* smem, uint32_t n, gu8* out, uint32_t cap,
                                int32_t* ret_slot, uint32_t* aux_slot, uint64_t* dbg, uint32_t lane,
                                bool progress_prio = true) {
    const Table<TT> T{smem};
    const uint64_t bound = (uint64_t)n + n / 255 + 16;
    const bool limited = cap < bound;  // lz4e_compress.c:553-560
    uint32_t op = 0, anchor = 0, ip = 0;
    [[maybe_unused]] uint32_t trn = 0;
    Stamps st;
    if (kStamps) st.start();

    if (n >= kMinLength) {
        const uint32_t mflimit = n - kMfLimit;
        const uint32_t matchlimit = n - kLastLiterals;
        const uint64_t lanes_below = (1ull << lane) - 1;
        const uint64_t lanes_above = lane >= 63 ? 0 : (~0ull << (lane + 1));
        const uint32_t xs[2] = {lane, 64 + lane};  // my two window positions

        // offset, match-length code and token (compress_block's emit_match)
        auto emit_match = [&](uint32_t tok, uint32_t tokhi, uint32_t off, uint32_t mc) -> bool {
            const uint32_t op_off = op;
            op += 2;
            if (limited && (uint64_t)op + 6 + (mc >> 8) > cap) return false;
            const uint32_t tokb = tokhi | (mc < 15 ? mc : 15);
            const uint32_t e1 = mc - 15;
            const uint32_t e1w = (mc >= 15 && e1 < 255) ? e1 : 0;
            if (lane == 0) {
                if (op_off == tok + 1) {
                    st32(out, tok, tokb | (off << 8) | (e1w << 24));
                } else {
                    out[tok] = (uint8_t)tokb;
                    st32(out, op_off, off | (e1w << 16));
                }
            }
            if (mc >= 15) {
                if (e1 < 255) {
                    op += 1;
                } else {
                    lockstep();
                    op += out_ext(out, op, e1, lane);
                }
            }
            return true;
        };

        bool rmode = false;
        uint32_t e = 1, s = 1, jb = 0, pf = 0;
        uint32_t prio_q = (n > 16384 && progress_prio) ? 4 : 5;
        uint32_t prio_next = prio_q == 5 ? ~0u : 0;
        M2 guess = {~0ull, ~0ull}, pprev = guess;
        uint32_t nB = ~0u, ndm1[2], ndv[2][kFwdW];
        auto preload = [&](uint32_t Bn) {
            if (Bn == nB) return;
            nB = Bn;
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h) {
                ndm1[h] = img.wld(Bn + xs[h] - 4);
#pragma unroll
                for (uint32_t i = 0; i < kFwdW; ++i) ndv[h][i] = img.wld(Bn + xs[h] + 4 * i);
            }
        };
        for (;;) {
            // ================= window setup =================================
            if (e >= prio_next) {
                const uint32_t q = (uint32_t)(((uint64_t)e * 4) / n);
                prio_next = q >= 4 ? ~0u : (uint32_t)(((uint64_t)(q + 1) * n + 3) / 4);
                if (q != prio_q) {
                    prio_q = q;
                    wave_prio_for(q);
                }
            }
            consume(pf);
            const uint32_t B = rmode ? e - 2 : e;
            uint32_t p[2], dm1[2], dv[2][kFwdW], hs[2], c0[2], rb[2];
            bool valid[2];
            const bool pre = B == nB;
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h) {
                p[h] = B + xs[h];
                valid[h] = p[h] <= mflimit;
                if (pre) {
                    dm1[h] = ndm1[h];
#pragma unroll
                    for (uint32_t i = 0; i < kFwdW; ++i) dv[h][i] = ndv[h][i];
                } else {
                    dm1[h] = img.wld(p[h] - 4);
#pragma unroll
                    for (uint32_t i = 0; i < kFwdW; ++i) dv[h][i] = img.wld(p[h] + 4 * i);
                }
                hs[h] = hash_val<TT>(((uint64_t)dv[h][1] << 32) | dv[h][0]);
                c0[h] = 0;
                rb[h] = p[h];
            }
            lockstep();  // the previous window's commit is in the table
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h)
                if (valid[h]) c0[h] = T.get(hs[h]);
            uint32_t em1[2], ev[2][kFwdW];
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h) {
                em1[h] = img.wld(c0[h] - 4);
#pragma unroll
                for (uint32_t i = 0; i < kFwdW; ++i) ev[h][i] = img.wld(c0[h] + 4 * i);
            }
            lockstep();
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h)
                if (valid[h]) T.put(hs[h], p[h]);
            lockstep();
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h)
                if (valid[h]) rb[h] = T.reread(hs[h]);
            // clash groups: valid positions whose read-back names the same
            // winning put (7-bit key rb - B, one ballot pair per key bit)
            M2 same[2] = {{0, 0}, {0, 0}};
            if (ballot(rb[0] != p[0]) | ballot(rb[1] != p[1])) {
                const M2 vmask = ballot2(valid[0], valid[1]);
                const uint32_t key[2] = {rb[0] - B, rb[1] - B};
                M2 m[2] = {vmask, vmask};
#pragma unroll
                for (uint32_t b = 0; b < 7; ++b) {
                    const M2 bb = ballot2((key[0] >> b) & 1, (key[1] >> b) & 1);
#pragma unroll
                    for (uint32_t h = 0; h < 2; ++h) m[h] = m[h] & (((key[h] >> b) & 1) ? bb : ~bb);
                }
#pragma unroll
                for (uint32_t h = 0; h < 2; ++h)
                    if (valid[h] && m2_popc(m[h]) >= 2) same[h] = m[h];
            }
            const M2 clash = ballot2(m2_any(same[0]), m2_any(same[1]));
            uint32_t lim[2], ml[2], bk[2];
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h) {
                lim[h] = matchlimit - p[h];
                ml[h] = 0;
                bk[h] = kNoBk;
                const bool dist_ok = (TT == kByU16) || (c0[h] + kMaxDistance >= p[h]);
                if (valid[h] && dist_ok) ml[h] = fwd_match(dv[h], ev[h], lim[h]);
                if (p[h] >= 4 && c0[h] >= 4) bk[h] = back4(dm1[h], em1[h]);
            }
            const M2 hitm = ballot2(ml[0] != 0, ml[1] != 0);
            M2 put = {0, 0};
            bool generic = false;
            // window position k against the earlier window position cl
            // (both wave-uniform), from the registers
            auto lanes_match = [&](uint32_t k, uint32_t cl, uint32_t& m, uint32_t& bb) {
                const uint32_t lk = matchlimit - (B + k);
                uint32_t ak[kFwdW], ac[kFwdW];
#pragma unroll
                for (uint32_t i = 0; i < kFwdW; ++i) {
                    const uint32_t v[2] = {dv[0][i], dv[1][i]};
                    ak[i] = pos_val(v, k);
                    ac[i] = pos_val(v, cl);
                }
                m = fwd_match(ak, ac, lk);
                bb = (B + k >= 4 && B + cl >= 4) ? back4(pos_val(dm1, k), pos_val(dm1, cl)) : kNoBk;
            };
            // my half-h position against the window position y (per lane),
            // the candidate's bytes re-read (L1)
            auto cand_match = [&](uint32_t h, uint32_t y, uint32_t& m, uint32_t& bb) {
                uint32_t g[kFwdW];
#pragma unroll
                for (uint32_t i = 0; i < kFwdW; ++i) g[i] = img.wld(y + 4 * i);
                const uint32_t gm1 = img.wld(y - 4);
                m = fwd_match(dv[h], g, lim[h]);
                bb = (p[h] >= 4 && y >= 4) ? back4(dm1[h], gm1) : kNoBk;
            };

            // ---- fast chain tables (compress_block's, per position) --------
            // fc: next rmode position (< 256) or kStop; fe: offset | literal
            // length << 16 | match length << 24; jv: last probe of the search.
            constexpr uint32_t kStop = 0x100;
            const int32_t lvs0 = (int32_t)mflimit - 1 - (int32_t)B;
            const M2 inlim0 = lvs0 < 0 ? M2{0, 0} : m2_below(lvs0 >= 127 ? 128u : (uint32_t)lvs0 + 1);
            auto chain_tables = [&](const uint32_t* vc, const uint32_t* vm, const uint32_t* vb,
                                    uint32_t* fc, uint32_t* fe, uint32_t* jv) {
                const M2 ah = ballot2(vm[0] != 0, vm[1] != 0) & inlim0;
                // candidate of each position, packed: offset | match (0xFF:
                // long) << 16 | back bytes << 24
                uint32_t pk[2], j[2];
#pragma unroll
                for (uint32_t h = 0; h < 2; ++h)
                    pk[h] = ((p[h] - vc[h]) & 0xFFFFu) | (((vm[h] & kLong) ? 0xFFu : vm[h]) << 16) |
                            (vb[h] << 24);
                {
                    // first hit among the step-1 probes after each position x:
                    // x + 1 .. x + 65 (P <= 64; a 64-position window never
                    // reaches further)
                    const uint64_t a0 = ah.lo & lanes_above, a1 = ah.hi & lanes_above;
                    const uint64_t h0 = ah.hi & (lane >= 62 ? ~0ull : ((4ull << lane) - 1));
                    j[0] = a0 ? ctz64(a0) : (h0 ? 64 + ctz64(h0) : 128);
                    j[1] = a1 ? 64 + ctz64(a1) : 128;
                }
                const uint32_t g0 = shfl(pk[0], j[0]), g1 = shfl(pk[1], j[0]);
                const uint32_t q[2] = {j[0] < 64 ? g0 : g1, shfl(pk[1], j[1])};
#pragma unroll
                for (uint32_t h = 0; h < 2; ++h) {
                    const uint32_t x = xs[h];
                    fc[h] = kStop;
                    fe[h] = 0;
                    jv[h] = x;
                    if (valid[h]) {
                        if (vm[h] != 0) {
                            if (!(vm[h] & kLong)) {
                                fc[h] = x + vm[h];
                                fe[h] = (p[h] - vc[h]) | (vm[h] << 24);
                            }
                        } else if (j[h] < 128) {
                            const uint32_t mlj = (q[h] >> 16) & 0xFFu, bkj = q[h] >> 24;
                            if (mlj != 0xFFu && bkj != kNoBk) {
                                const uint32_t off = q[h] & 0xFFFFu, cj = B + j[h] - off;
                                const uint32_t room = j[h] - x < cj ? j[h] - x : cj;
                                const uint32_t cu = bkj < room ? bkj : room;
                                if (!(cu == 4 && room > 4)) {
                                    fc[h] = j[h] + mlj;
                                    fe[h] = off | ((j[h] - cu - x) << 16) | ((mlj + cu) << 24);
                                    jv[h] = j[h];
                                }
                            }
                        }
                    }
                }
            };
            uint32_t fc0[2] = {kStop, kStop}, fe0[2] = {0, 0}, jv0[2] = {xs[0], xs[1]};
            bool have0 = false;
            // touch [B + 128, B + 384): the next window's loads hit cache
            pf = img.wld(B + 128 + 4 * lane);
            if (kStamps) { st.cnt[0]++; st.lap(kPhSearch); }

            // ================= walk =========================================
            for (;;) {
                if (rmode && !limited) {
                    // ---- fast chain with the clash fixpoint (compress_block) --
                    if (kStamps) st.lap(kPhStripe);
                    const uint32_t ks = e - B;
                    uint32_t k = ks, nev = 0, evl = 0;
                    M2 evm = {0, 0}, pch = {0, 0};
                    uint32_t fc[2] = {kStop, kStop}, fe[2] = {0, 0}, jv[2] = {xs[0], xs[1]};
                    if (ks < 128) {
                        const bool dyn = m2_any(clash & ~m2_below(ks));
                        if (!dyn) {
                            if (!have0) {
                                chain_tables(c0, ml, bk, fc0, fe0, jv0);
                                have0 = true;
                            }
#pragma unroll
                            for (uint32_t h = 0; h < 2; ++h) {
                                fc[h] = fc0[h];
                                fe[h] = fe0[h];
                                jv[h] = jv0[h];
                            }
                        }
                        M2 Pg = put | m2_bit(ks - 2) | m2_bit(ks) | (guess & ~m2_below(ks));
                        constexpr uint32_t kMaxPass = 6;
                        for (uint32_t pass = 0;; ++pass) {
                            if (kStamps) st.cnt[2]++;
                            if (dyn) {
                                uint32_t vc[2], vm[2], vb[2];
#pragma unroll
                                for (uint32_t h = 0; h < 2; ++h) {
                                    vc[h] = c0[h];
                                    vm[h] = ml[h];
                                    vb[h] = bk[h];
                                    const M2 pm = same[h] & Pg & below_me(h, lanes_below);
                                    if (half_bit(clash, h, lane) && m2_any(pm)) {
                                        const uint32_t cl = (uint32_t)m2_top(pm);
                                        vc[h] = B + cl;
                                        cand_match(h, B + cl, vm[h], vb[h]);
                                    }
                                }
                                chain_tables(vc, vm, vb, fc, fe, jv);
                            }
                            if (kStamps) st.lap(kPhCount);
                            // fc^2, fc^3, fc^4 (a position past the window or
                            // stopped stays put): four links per walk step
                            const uint32_t FC = pk2(fc[0], fc[1]);
                            uint32_t J2[2], J3[2], J4[2];
#pragma unroll
                            for (uint32_t h = 0; h < 2; ++h) {
                                const uint32_t g = pk_shfl(FC, fc[h]);
                                J2[h] = fc[h] < 128 ? g : fc[h];
                            }
                            const uint32_t J2P = pk2(J2[0], J2[1]);
#pragma unroll
                            for (uint32_t h = 0; h < 2; ++h) {
                                const uint32_t g2 = pk_shfl(FC, J2[h]), g3 = pk_shfl(J2P, J2[h]);
                                J3[h] = J2[h] < 128 ? g2 : J2[h];
                                J4[h] = J2[h] < 128 ? g3 : J2[h];
                            }
                            const uint32_t J3P = pk2(J3[0], J3[1]), J4P = pk2(J4[0], J4[1]);
                            k = ks;
                            evm = {0, 0};
                            while (k < 128) {
                                const uint32_t l = k & 63, sh = (k >> 2) & 16;
                                const uint32_t x1 = (lane_val(FC, l) >> sh) & 0xFFFFu;
                                const uint32_t x2 = (lane_val(J2P, l) >> sh) & 0xFFFFu;
                                const uint32_t x3 = (lane_val(J3P, l) >> sh) & 0xFFFFu;
                                const uint32_t x4 = (lane_val(J4P, l) >> sh) & 0xFFFFu;
                                if (x1 & kStop) break;
                                evm = evm | m2_bit(k);
                                if (x1 >= 128) { k = x1; break; }
                                if (x2 & kStop) { k = x1; break; }
                                evm = evm | m2_bit(x1);
                                if (x2 >= 128) { k = x2; break; }
                                if (x3 & kStop) { k = x2; break; }
                                evm = evm | m2_bit(x2);
                                if (x3 >= 128) { k = x3; break; }
                                if (x4 & kStop) { k = x3; break; }
                                evm = evm | m2_bit(x3);
                                k = x4;
                            }
                            nev = m2_popc(evm);
                            // the chain's puts: e-2 and e of every event, the
                            // probes (l, jv(l)] of its searches
                            {
                                const uint32_t JVP = pk2(jv[0], jv[1]);
                                bool pr[2];
#pragma unroll
                                for (uint32_t h = 0; h < 2; ++h) {
                                    const int32_t lb = m2_top(evm & below_me(h, lanes_below));
                                    const uint32_t jl = pk_shfl(JVP, lb < 0 ? xs[h] : (uint32_t)lb);
                                    pr[h] = lb >= 0 && xs[h] <= jl;
                                }
                                pch = ballot2(pr[0], pr[1]) | evm | m2_shr2(evm);
                            }
                            if (!dyn) break;
                            const M2 Pn = put | pch;
                            const M2 U = pch & ~m2_shr2(evm);
                            bool bad[2];
#pragma unroll
                            for (uint32_t h = 0; h < 2; ++h) {
                                const M2 mem = same[h] & below_me(h, lanes_below);
                                bad[h] = half_bit(U, h, lane) && m2_top(mem & Pg) != m2_top(mem & Pn);
                            }
                            if (!m2_any(ballot2(bad[0], bad[1]))) break;  // fixpoint
                            if (pass + 1 == kMaxPass) {                   // give up: exact walk
                                nev = 0;
                                k = ks;
                                pch = {0, 0};
                                break;
                            }
                            Pg = Pn | (k >= 128 ? M2{0, 0} : ~m2_below(k));
                        }
                        put = put | pch;
                        // evl: lane q < nev holds the window position of event q
                        const uint32_t n0 = popc64(evm.lo);
                        const uint32_t r0 =
                            push_lane(xs[0], half_bit(evm, 0, lane) ? popc64(evm.lo & lanes_below) : 63);
                        const uint32_t r1 = push_lane(
                            xs[1], half_bit(evm, 1, lane) ? n0 + popc64(evm.hi & lanes_below) : 63);
                        evl = lane < n0 ? r0 : r1;
                    }
                    if (kStamps) st.lap(kPhLit);
                    if (nev) {
                        // emit the nev sequences at once (lz4e_compress.c:352-453)
                        const uint32_t fi = lane < nev ? evl : 0;
                        const uint32_t fa = shfl(fe[0], fi), fb = shfl(fe[1], fi);
                        const uint32_t f = fi < 64 ? fa : fb;
                        const uint32_t L = (f >> 16) & 0xFF, mc = (f >> 24) - 4;
                        const uint32_t hdr = L >= 15 ? 2 : 1;
                        const uint32_t size = lane < nev ? hdr + L + 2 + (mc >= 15 ? 1 : 0) : 0;
                        const uint32_t o = op + wave_incl_add(size) - size;
                        if (lane < nev) {
                            out[o] = (uint8_t)(((L < 15 ? L : 15) << 4) | (mc < 15 ? mc : 15));
                            if (L >= 15) out[o + 1] = (uint8_t)(L - 15);
                            out[o + hdr + L] = (uint8_t)f;
                            out[o + hdr + L + 1] = (uint8_t)(f >> 8);
                            if (mc >= 15) out[o + hdr + L + 2] = (uint8_t)(mc - 15);
                        }
                        // literal byte of position x: run of the last event s <= x
#pragma unroll
                        for (uint32_t h = 0; h < 2; ++h) {
                            const int32_t sx = m2_top(evm & below_me(h, lanes_below | (1ull << lane)));
                            const uint32_t su = sx < 0 ? 0 : (uint32_t)sx;
                            const uint32_t qi = m2_popc(evm & m2_below(su));
                            const uint32_t Lq = shfl(L, qi), dq = shfl(o + hdr, qi);
                            if (sx >= 0 && xs[h] - su < Lq) out[dq + xs[h] - su] = (uint8_t)dv[h][0];
                        }
                        op = lane_val(o + size, nev - 1);
                        e = B + k;
                        anchor = e;
                        if (kStamps) { st.cnt[1] += nev; st.cnt[3] += nev << 16; st.lap(kPhTail); }
                        if (e > mflimit) {  // :456-457
                            ip = e;
                            goto last_literals;
                        }
                    }
                }
                if (kStamps && rmode && !limited) { st.cnt[3]++; st.lap(kPhLit); }
                if (rmode) {
                    // ---- fill table at e-2, test e (lz4e_compress.c:461-493) ----
                    const uint32_t k = e - B;
                    if (k > 127) break;
                    const M2 prior = put | m2_bit(k - 2);
                    uint32_t c, m;
                    bool grp = false;
                    uint32_t cl = 0;
                    if (m2_any(clash & m2_bit(k))) {
                        const uint32_t l = k & 63;
                        const M2 sk = k < 64 ? M2{lane_val64(same[0].lo, l), lane_val64(same[0].hi, l)}
                                             : M2{lane_val64(same[1].lo, l), lane_val64(same[1].hi, l)};
                        const int32_t t = m2_top(sk & prior & m2_below(k));
                        grp = t >= 0;
                        cl = (uint32_t)t;
                    }
                    if (grp) {
                        c = B + cl;
                        uint32_t bb;
                        lanes_match(k, cl, m, bb);
                    } else {
                        c = pos_val(c0, k);
                        m = pos_val(ml, k);
                    }
                    put = prior | m2_bit(k);
                    if (kStamps) st.lap(kPhCount);
                    if (m == 0) {
                        // no match at e: search from e + 1 (:496-497)
                        rmode = false;
                        s = e = e + 1;
                        jb = 0;
                        continue;
                    }
                    uint32_t t = m & ~kLong;
                    if (m & kLong) t = count_from(img, e, c, kFwd, matchlimit, lane);
                    LZ4E_TR(2, e, ((uint64_t)c << 32) | t);
                    const uint32_t tok = op++;
                    if (!emit_match(tok, 0, e - c, t - 4)) goto fail;
                    if (kStamps) st.cnt[1]++;
                    e += t;
                    anchor = e;
                    if (e > mflimit) {  // :456-457
                        ip = e;
                        goto last_literals;
                    }
                    continue;
                }

                // ---- search: probes P = jb + (k - k0) at positions k >= k0 ----
                const uint32_t k0 = e - B;
                if (k0 > 127) break;
                const uint32_t kmax = k0 + 64 - jb < 127 ? k0 + 64 - jb : 127;  // P <= 64: step 1
                // probe q runs iff q + 1 <= mflimit (:301-302)
                const int32_t lvs = (int32_t)mflimit - 1 - (int32_t)B;
                if (lvs < (int32_t)k0) {
                    ip = jb ? e - 1 : s;  // the last probe that ran
                    goto last_literals;
                }
                const uint32_t lastv = (uint32_t)lvs < kmax ? (uint32_t)lvs : kmax;
                const M2 rng = m2_range(k0, lastv);
                const M2 A = hitm & ~clash & rng;
                M2 CL = clash & rng;
                if (m2_any(A)) CL = CL & m2_below(m2_ctz(A));
                uint32_t hk = 128, c = 0, m = 0, b = kNoBk;
                // a clash probe's candidate: the latest member of its group
                // put before it (the window's puts, this search's earlier
                // probes), else c0
                uint32_t vc[2] = {c0[0], c0[1]}, vm[2] = {ml[0], ml[1]}, vb[2] = {bk[0], bk[1]};
                if (m2_any(CL)) {
                    const M2 prior0 = put | ~m2_below(k0);
#pragma unroll
                    for (uint32_t h = 0; h < 2; ++h) {
                        const M2 pm = same[h] & prior0 & below_me(h, lanes_below);
                        if (half_bit(CL, h, lane) && m2_any(pm)) {
                            const uint32_t cl = (uint32_t)m2_top(pm);
                            vc[h] = B + cl;
                            cand_match(h, B + cl, vm[h], vb[h]);
                        }
                    }
                }
                const M2 CA = CL | A;
                const M2 H = ballot2(half_bit(CA, 0, lane) && vm[0] != 0, half_bit(CA, 1, lane) && vm[1] != 0);
                if (m2_any(H)) {
                    hk = m2_ctz(H);
                    c = pos_val(vc, hk);
                    m = pos_val(vm, hk);
                    b = pos_val(vb, hk);
                }
                if (hk == 128) {
                    // no hit among this window's probes: all of them put
                    put = put | rng;
                    jb += lastv - k0 + 1;
                    e = B + lastv + 1;
                    if (lastv < kmax) {  // the next probe would pass mflimit
                        ip = B + lastv;
                        goto last_literals;
                    }
                    if (jb > 64) {  // skip steps > 1 from here: generic search
                        generic = true;
                        break;
                    }
                    continue;  // next window
                }
                put = put | m2_range(k0, hk);
                if (kStamps) st.lap(kPhStripe);
                const uint32_t q = B + hk;
                // catch up (lz4e_compress.c:339-349)
                const uint32_t room = q - anchor < c ? q - anchor : c;
                uint32_t cu;
                if (b == kNoBk) {
                    cu = back_from(img, q, c, room);
                } else {
                    cu = b < room ? b : room;
                    if (cu == 4 && room > 4) cu += back_from(img, q - 4, c - 4, room - 4);
                }
                const uint32_t ipm = q - cu, cand = c - cu;
                uint32_t t = m & ~kLong;
                if (m & kLong) t = count_from(img, q, c, kFwd, matchlimit, lane);
                t += cu;
                LZ4E_TR(2, ipm, ((uint64_t)cand << 32) | t);
                // literals [anchor, ipm) (lz4e_compress.c:352-382)
                const uint32_t L = ipm - anchor;
                const uint32_t tok = op++;
                if (limited && (uint64_t)op + L + 8 + L / 255 > cap) goto fail;
                uint32_t tokhi;
                if (L >= 15) {
                    tokhi = 0xF0;
                    op += out_ext(out, op, L - 15, lane);
                } else {
                    tokhi = L << 4;
                }
                if (anchor >= B) {
                    // the run lies in the window: position a0 + 4i stores bytes 4i..4i+3
#pragma unroll
                    for (uint32_t h = 0; h < 2; ++h) {
                        const uint32_t r = xs[h] - (anchor - B);
                        if ((r & 3) == 0 && r < L) st32(out, op + r, dv[h][0]);
                    }
                } else {
                    out_copy(out, op, img, anchor, L, lane);
                }
                op += L;
                lockstep();  // the offset overwrites the copy's spare bytes
                if (!emit_match(tok, tokhi, ipm - cand, t - 4)) goto fail;
                if (kStamps) { st.cnt[1]++; st.lap(kPhTail); }
                e = ipm + t;
                anchor = e;
                rmode = true;
                if (e > mflimit) {
                    ip = e;
                    goto last_literals;
                }
            }
            if (kStamps) st.lap(kPhStripe);

            // ================= commit the window's puts =====================
            if (!generic) preload(rmode ? e - 2 : e);
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h) {
                if (valid[h]) {
                    const M2 pg = same[h] & put;
                    bool writer;
                    uint32_t v;
                    if (!m2_any(same[h])) {
                        writer = true;
                        v = half_bit(put, h, lane) ? p[h] : c0[h];
                    } else if (m2_any(pg)) {
                        writer = (int32_t)xs[h] == m2_top(pg);
                        v = p[h];
                    } else {
                        writer = xs[h] == m2_ctz(same[h]);
                        v = c0[h];
                    }
                    if (writer) T.put(hs[h], v);
                }
            }
            {
                const M2 R = {~7ull, ~0ull};
                const uint32_t mp = m2_popc((put ^ pprev) & R), mo = m2_popc(~put & R);
                guess = mp < mo ? put : M2{~0ull, ~0ull};
                pprev = put;
            }
            if (kStamps) st.lap(kPhRematch);
            if (!generic) continue;

            // ================= generic search (probes P >= 65) ==============
            // (compress_block's, one probe per lane)
            {
                uint32_t pbase = jb, qh, ch;
                for (;;) {
                    const uint32_t P = pbase + lane;
                    const uint32_t qq = s + (uint32_t)probe_offset(P);
                    const bool pv = (uint64_t)qq + probe_step(P) <= mflimit;
                    const uint64_t vmask = ballot(pv);
                    if (vmask == 0) {
                        ip = s + (uint32_t)probe_offset(pbase - 1);
                        goto last_literals;
                    }
                    const uint32_t q = pv ? qq : s;
                    uint64_t v;
                    if constexpr (TT == kByU32) v = img.ld64(q);
                    else v = img.ld32(q);
                    const uint32_t vq = (uint32_t)v;
                    const uint32_t hq = hash_val<TT>(v);
                    uint32_t g0 = 0, grb = q;
                    lockstep();
                    if (pv) g0 = T.get(hq);
                    lockstep();
                    if (pv) T.put(hq, q);
                    lockstep();
                    if (pv) grb = T.reread(hq);
                    const uint64_t gcm = ballot(grb != q);
                    uint64_t gsame = 0;
                    uint32_t gc = g0;
                    if (gcm) {
                        uint64_t todo = gcm;
                        do {
                            const uint32_t hg = lane_val(hq, ctz64(todo));
                            const uint64_t mm = ballot(pv && hq == hg);
                            if (hq == hg) gsame = mm;
                            todo &= ~mm;
                        } while (todo);
                        const uint64_t below = gsame & lanes_below;
                        const uint32_t qp =
                            shfl(q, below ? 63 - (uint32_t)__builtin_clzll(below) : lane);
                        if (below) gc = qp;
                    }
                    bool hit = false;
                    if (pv) {
                        const bool dist_ok = (TT == kByU16) || (gc + kMaxDistance >= q);
                        hit = dist_ok && img.ld32(gc) == vq;
                    }
                    const uint64_t hm = ballot(hit);
                    const uint32_t klast = hm ? ctz64(hm) : popc64(vmask) - 1;
                    if (pv) {
                        if (gcm == 0) {
                            if (lane > klast) T.put(hq, g0);
                        } else {
                            const uint64_t upto = klast >= 63 ? ~0ull : ((2ull << klast) - 1);
                            if (lane <= klast) {
                                if ((gsame & upto & ~((2ull << lane) - 1)) == 0) T.put(hq, q);
                            } else if ((gsame & upto) == 0) {
                                T.put(hq, g0);
                            }
                        }
                    }
                    if (hm) {
                        qh = lane_val(q, klast);
                        ch = lane_val(gc, klast);
                        break;
                    }
                    if (vmask != ~0ull) {
                        ip = lane_val(q, klast);  // the last probe that ran
                        goto last_literals;
                    }
                    pbase += kWave;
                }
                const uint32_t room = qh - anchor < ch ? qh - anchor : ch;
                const uint32_t cu = back_from(img, qh, ch, room);
                const uint32_t ipm = qh - cu, cand = ch - cu;
                const uint32_t t = count_from(img, qh, ch, 4, matchlimit, lane) + cu;
                LZ4E_TR(2, ipm, ((uint64_t)cand << 32) | t);
                const uint32_t L = ipm - anchor;
                const uint32_t tok = op++;
                if (limited && (uint64_t)op + L + 8 + L / 255 > cap) goto fail;
                uint32_t tokhi;
                if (L >= 15) {
                    tokhi = 0xF0;
                    op += out_ext(out, op, L - 15, lane);
                } else {
                    tokhi = L << 4;
                }
                out_copy(out, op, img, anchor, L, lane);
                op += L;
                lockstep();
                if (!emit_match(tok, tokhi, ipm - cand, t - 4)) goto fail;
                if (kStamps) { st.cnt[1]++; st.lap(kPhLit); }
                e = ipm + t;
                anchor = e;
                rmode = true;
                if (e > mflimit) {
                    ip = e;
                    goto last_literals;
                }
            }
        }
    }

last_literals: {
        // lz4e_compress.c:500-530
        const uint32_t R = n - anchor;
        if (limited && (uint64_t)op + R + 1 + (R + 240) / 255 > cap) goto fail;
        if (R >= 15) {
            if (lane == 0) out[op] = 0xF0;
            op += 1;
            op += out_ext(out, op, R - 15, lane);
        } else {
            if (lane == 0) out[op] = (uint8_t)(R << 4);
            op += 1;
        }
        out_copy_exact(out, op, img, anchor, R, lane);
        if (lane == 0) {
            *ret_slot = (int32_t)(op + R);
            if (aux_slot) {
                aux_slot[0] = ip;
                aux_slot[1] = R;
            }
        }
        if (kStamps) {
            st.lap(kPhTail);
            if (lane == 0 && dbg) {
                for (int i = 0; i < 6; ++i) dbg[i] = st.acc[i];
                dbg[6] = ((uint64_t)st.cnt[1] << 32) | st.cnt[0];
                dbg[7] = ((uint64_t)st.cnt[3] << 32) | st.cnt[2];
            }
        }
        return;
    }
fail:
    if (lane == 0) {
        *ret_slot = 0;
        if (aux_slot) {
            aux_slot[0] = 0;
            aux_slot[1] = 0;
        }
    }
}
