// Speculative parallel frontier walk (N <= 32, fresh state).
//
// The frontier recurrence C_{r+1} = F(C_r) (hge_kernels.hip, k_rounds_walk;
// DivideRounds, hashgraph.go:211-305 and 573-588) is a deterministic map of the
// whole frontier vector, so two walks that ever reach the same vector coincide
// from then on.  Measured on random gossip, a walk started from a guessed
// frontier (chain positions in proportion, floor(len_c * w / nw)) lands on the
// true trajectory within ~1-60 steps.  So nw walkers start at once, walker w
// from guess w (walker 0 from the true start C_0), each one wave walking from
// LDS exactly like k_rounds_walk, and each publishing its rows (local round
// numbering, row 0 = its start) to a history buffer in HBM.  While wave 0
// walks, waves 1-3 of the same workgroup compare the walker's newest row with
// the published rows of the next WIN walkers; the first equal row (walker t,
// row b) is a merge: the walker stops, since its future is walker t's from row
// b on.  k_walk_join then follows the merges from walker 0 (whose rows are true
// by construction) and copies the true rows into C with global round numbers.
// Nothing is assumed: a walker that reaches its history capacity without a
// merge ends the chain there, and the sequential k_rounds_walk resumes from the
// last true row (k_walk_join writes its round to *resume, -1 = complete), so the
// result is identical to the sequential walk in every case; only the time
// depends on how soon the walkers merge.
//
// Cross-workgroup hand-off without fences ("data is the flag", as k_rounds_coop):
// every history entry is 64 bits, (launch epoch << 32) | position, written by
// the owner lane as soon as the step computes it with a relaxed agent-scope
// (write-through) store, so publishing costs the walk no wait.  A checker
// compares whole tagged words with relaxed agent-scope loads: an entry that is
// stale (older epoch) or not yet visible never equals a current one, so it can
// only delay a merge, never fake one.  Each row index is written once per
// launch.  Lane 0 also stores a progress hint (rows so far) that bounds the
// scan.  No workgroup ever waits on another, so the launch needs no co-residency.
namespace hge {

__device__ __forceinline__ int s_r0_rows(int r, int st) { return r + 1; }

template <int NPC, int LPC, int B>
__global__ void __launch_bounds__(1024) k_walk_spec(Tables t, const uint16_t* FSS,
                                                    const int32_t* len, int nw, int Hcap,
                                                    uint64_t* H, int32_t* hn, int32_t* hp,
                                                    int4* res, uint32_t epoch, int nchk,
                                                    int nsleep, uint64_t* wdbg) {
  constexpr int VPL = NPC / LPC;
  constexpr int RB = 64;       // rows per walk segment (the sC buffer the checkers read)
  constexpr int Q8 = NPC / 8;  // int4 loads per fss row
  constexpr int BR = B + 1;    // block rows per chain: B staged + the 0xFFFF row
  constexpr int WIN = 6;       // later walkers a walker checks against
  // nchk checker threads (waves 1 .. nchk/64), each pausing nsleep x 64 cycles
  // between polls; the rest prefetch
  const int NCHK = nchk;
  static_assert(NPC * LPC == 64, "one wave walks");
  int pf = 0;  // prefetch sink
  __shared__ __attribute__((aligned(16))) uint16_t blk[NPC * BR * NPC];  // [d][row][c]
  __shared__ __attribute__((aligned(16))) int sA[NPC];
  __shared__ int sP[NPC], sBase[NPC], sLen[NPC], sC[RB * NPC];
  __shared__ int s_r, s_lv, s_status, s_len, s_cur, s_wdone, s_mflag;
  __shared__ unsigned long long s_mkey;
  const int N = t.N, SM = t.SM;
  const int tid = threadIdx.x, T = blockDim.x;
  const int w = blockIdx.x;
  uint64_t d_t0 = 0, d_rs = 0, d_nrs = 0, d_tw = 0;  // wdbg: cycles, restage cycles, restages
  if (wdbg && tid == 0) d_t0 = stamp();
  uint64_t* Hw = H + (size_t)w * Hcap * N;
  const uint64_t tag = (uint64_t)epoch << 32;
  if (tid < NPC) {
    const int c = tid;
    int P = INF32, ln = 0;
    if (c < N) {
      ln = len[c];
      if (ln > 0) P = (int)((int64_t)ln * w / nw);  // walker 0: position 0 = C_0
      __hip_atomic_store(Hw + c, tag | (uint32_t)P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    sP[c] = P;
    sLen[c] = ln;
  }
  for (int i = tid; i < NPC * NPC; i += T) blk[((i / NPC) * BR + B) * NPC + (i % NPC)] = 0xFFFF;
  if (tid == 0) {
    s_r = 0;
    s_lv = 1;
    s_status = 0;
    s_len = 0;
    s_mflag = 0;
    s_mkey = ~0ull;
  }
  if (tid == 0) __hip_atomic_store(hp + w, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  for (;;) {
    const int r0 = s_r;
    if (wdbg && tid == 0) d_tw = stamp();
    if (s_lv) {
      if (wdbg && tid == 0) d_nrs++;
      // restage: uint16 fss rows [P_d, P_d + B) of every chain (as k_rounds_walk)
      constexpr int ITEMS = NPC * B * Q8;
      constexpr int PER = (ITEMS + 1023) / 1024;
      int4 vals[PER];
#pragma unroll
      for (int m = 0; m < PER; m++) {
        const int item = tid + m * 1024;
        const int d = item / (B * Q8);
        const int rem = item - d * (B * Q8);
        const int k = rem / Q8, q8 = rem - k * Q8;
        int4 v4 = make_int4(-1, -1, -1, -1);
        if (item < ITEMS && d < N && sP[d] != INF32 && sP[d] + k < sLen[d])
          v4 = *(const int4*)(FSS + ((size_t)d * t.ccap + sP[d] + k) * NPC + 8 * q8);
        vals[m] = v4;
      }
#pragma unroll
      for (int m = 0; m < PER; m++) {
        const int item = tid + m * 1024;
        if (item >= ITEMS) break;
        const int d = item / (B * Q8);
        const int rem = item - d * (B * Q8);
        const int k = rem / Q8, q8 = rem - k * Q8;
        *(int4*)&blk[(d * BR + k) * NPC + 8 * q8] = vals[m];
      }
      if (tid < NPC) {
        sBase[tid] = sP[tid];
        sA[tid] = sP[tid] == INF32 ? B : 0;
      }
    }
    if (tid == 0) {
      s_cur = r0;
      s_wdone = 0;
    }
    __syncthreads();
    if (wdbg && tid == 0) d_rs += stamp() - d_tw;
    if (tid < 64) {
      // ---- wave 0 walks (the k_rounds_walk step with no known rows)
      const int lane = tid;
      const int c = lane / LPC, q = lane - (lane / LPC) * LPC;
      const bool act = c < N;
      const int ln = sLen[c];
      const int base_c = sBase[c];
      const int qo = (SM - 1) / VPL, ko = (SM - 1) - qo * VPL;
      const bool owner = act && q == qo;
      int gb[VPL];
#pragma unroll
      for (int k = 0; k < VPL; k++) gb[k] = 2 * (((q * VPL + k) * BR) * NPC + c);
      int myP = sP[c];
      int r = r0, st = 0;  // st: 1 merged, 2 end of the graph, 3 history full
      bool lvb = false;
      const int rcap1 = Hcap - 1;
      // a segment ends before the ring wraps onto rows not yet published
      const int rend = min(r0 + RB - 2, rcap1);
      for (;;) {
        if (r >= rend) {
          if (r >= rcap1) st = 3;
          break;
        }
        int Av[VPL], v[VPL];
#pragma unroll
        for (int k = 0; k < VPL; k++) Av[k] = sA[q * VPL + k];
        const int mf = __hip_atomic_load(&s_mflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
        for (int k = 0; k < VPL; k++)
          v[k] = *(const uint16_t*)((const char*)blk + gb[k] + Av[k] * (2 * NPC));
        __builtin_amdgcn_sched_barrier(0);
        if (mf) {
          st = 1;
          break;
        }
        int sel;
        if constexpr (NPC == 16 && VPL == 4) {
          sel = net16_packed((uint32_t)v[0] | ((uint32_t)v[2] << 16),
                             (uint32_t)v[1] | ((uint32_t)v[3] << 16), q, ko);
        } else {
#pragma unroll
          for (int size = 2; size <= NPC; size <<= 1) {
            if (size <= VPL) {
#pragma unroll
              for (int k = 0; k < VPL; k++) {
                const int k2 = k ^ (size - 1);
                if (k2 > k) {
                  const int a = v[k], b = v[k2];
                  v[k] = min(a, b);
                  v[k2] = max(a, b);
                }
              }
            } else {
              const bool lower = (q & ((size >> 1) / VPL)) == 0;
              int o[VPL];
#pragma unroll
              for (int k = 0; k < VPL; k++) o[k] = dpp_flip(size / VPL - 1, v[VPL - 1 - k]);
#pragma unroll
              for (int k = 0; k < VPL; k++) v[k] = lower ? min(v[k], o[k]) : max(v[k], o[k]);
            }
#pragma unroll
            for (int stride = size >> 2; stride > 0; stride >>= 1) {
              if (stride < VPL) {
#pragma unroll
                for (int k = 0; k < VPL; k++) {
                  const int k2 = k ^ stride;
                  if (k2 > k) {
                    const int a = v[k], b = v[k2];
                    v[k] = min(a, b);
                    v[k2] = max(a, b);
                  }
                }
              } else {
                const bool lower = (q & (stride / VPL)) == 0;
#pragma unroll
                for (int k = 0; k < VPL; k++) {
                  const int o = dpp_flip(stride / VPL, v[k]);
                  v[k] = lower ? min(v[k], o) : max(v[k], o);
                }
              }
            }
          }
          sel = v[0];
#pragma unroll
          for (int k = 1; k < VPL; k++) sel = (k == ko) ? v[k] : sel;
        }
        const int cand = sel < ln ? sel : INF32;
        const int nxt = myP == INF32 ? INF32 : cand;
        myP = nxt;
        const int rowA = nxt == INF32 ? B : nxt - base_c;
        if (owner) {
          sP[c] = nxt;
          sA[c] = min(rowA, B);
          sC[(r + 1) % RB * NPC + c] = nxt;  // ring of rows; the checker waves publish them
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const bool alive_l = owner && nxt != INF32;
        const uint64_t alive = __builtin_amdgcn_ballot_w64(alive_l);
        // a walker off the true trajectory can step BACK along a chain (the map is
        // monotone, but a guessed start is not below its image): that member
        // leaves its block too
        const uint64_t lv = __builtin_amdgcn_ballot_w64(alive_l && (rowA >= B || rowA < 0));
        if (alive == 0) {
          st = 2;
          break;
        }
        r++;
        // the row r is complete in sC (one wave's LDS writes land in order): hand
        // it to the checker waves
        if (lane == 0) __hip_atomic_store(&s_cur, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (lv != 0) {
          lvb = true;
          break;
        }
      }
      if (lane == 0) {
        s_r = r;
        s_lv = lvb;
        s_status = st;
        s_len = r + 1;  // end / full: rows 0..r are this walker's rows
        __hip_atomic_store(&s_wdone, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    } else if (tid < 64 + NCHK) {
      // ---- waves 1-7 look for the walker's newest row among the rows of
      //      walkers w+1 .. w+WIN (flattened over (walker, row))
      const int ct = tid - 64;
      int checked = r0;
      for (;;) {
        // acquire: the s_cur load below may not move above it (the final pass must
        // see the final row)
        const int wd = __hip_atomic_load(&s_wdone, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        const int rr = __hip_atomic_load(&s_cur, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (rr > checked) {
          // publish rows checked+1 .. rr (the walker itself never stores to HBM).
          // Entry (q, c) belongs to thread (q*N + c) mod NCHK whatever rows the
          // other checker threads have seen, so every entry is published once.
          const int g0 = (checked + 1) * N, g1 = (rr + 1) * N;
          for (int g = g0 + ((ct - g0) % NCHK + NCHK) % NCHK; g < g1; g += NCHK) {
            const int q = g / N, c = g - q * N;
            __hip_atomic_store(Hw + (size_t)q * N + c, tag | (uint32_t)sC[q % RB * NPC + c],
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          if (ct == 0) __hip_atomic_store(hp + w, rr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (rr > checked &&
            !__hip_atomic_load(&s_mflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
          // the newest row stays in LDS (registers are scarce at 1024 threads)
          const int* svr = sC + rr % RB * NPC;
          const uint64_t sv0 = tag | (uint32_t)svr[0];
          int cnt[WIN];
#pragma unroll
          for (int k = 0; k < WIN; k++)
            cnt[k] = w + 1 + k < nw
                         ? 1 + __hip_atomic_load(hp + w + 1 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                         : 0;
          // rows of the WIN later walkers flattened: item i -> (walker k, row b);
          // first columns of up to MAXI items per thread in flight at once, full
          // rows only for the items whose first column matches
          constexpr int MAXI = 2;
          int tot = 0;
#pragma unroll
          for (int k = 0; k < WIN; k++) tot += cnt[k];
          for (int i0 = ct; i0 < tot; i0 += MAXI * NCHK) {
            int ik[MAXI], ib[MAXI];
            uint64_t c0[MAXI];
#pragma unroll
            for (int m = 0; m < MAXI; m++) {
              int i = i0 + m * NCHK, k = 0;
              ik[m] = -1;
              if (i < tot) {
                while (i >= cnt[k]) i -= cnt[k++];
                ik[m] = k + 1;
                ib[m] = i;
              }
            }
#pragma unroll
            for (int m = 0; m < MAXI; m++)
              c0[m] = ik[m] > 0 ? __hip_atomic_load(H + ((size_t)(w + ik[m]) * Hcap + ib[m]) * N,
                                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                : 0;
#pragma unroll
            for (int m = 0; m < MAXI; m++) {
              if (ik[m] > 0 && c0[m] == sv0) {
                // rare: the first column matches, compare the rest one by one
                const uint64_t* row = H + ((size_t)(w + ik[m]) * Hcap + ib[m]) * N;
                bool eq = true;
                for (int c = 1; c < N && eq; c++)
                  eq = __hip_atomic_load(row + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                       (tag | (uint32_t)svr[c]);
                if (eq) {
                  atomicMin(&s_mkey, ((unsigned long long)rr << 40) |
                                         ((unsigned long long)ik[m] << 32) | (unsigned long long)ib[m]);
                  __hip_atomic_store(&s_mflag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
              }
            }
          }
          checked = rr;
        }
        if (wd) break;
        for (int z = 0; z < nsleep; z++) __builtin_amdgcn_s_sleep(1);
      }
    } else {
      // ---- the other waves pull the rows after every block into L2 (as k_rounds_walk)
      constexpr int RPL = 128 / (2 * NPC);
      constexpr int LPCH = B / RPL;
      for (int item = tid - 64 - NCHK; item < NPC * LPCH; item += T - 64 - NCHK) {
        const int d = item / LPCH, k = (item - d * LPCH) * RPL;
        if (d < N && sBase[d] != INF32 && sBase[d] + B + k < sLen[d])
          pf ^= *(const int*)(FSS + ((size_t)d * t.ccap + sBase[d] + B + k) * NPC);
      }
    }
    __syncthreads();
    const int fin = s_status;
    if (fin) {
      if (tid == 0) {
        // rows published: 0..r
        hn[w] = s_r0_rows(s_r, fin);
        if (wdbg) {
          wdbg[4 * w] = stamp() - d_t0;
          wdbg[4 * w + 1] = d_rs;
          wdbg[4 * w + 2] = d_nrs;
          wdbg[4 * w + 3] = s_r;
        }
        if (fin == 1) {
          const unsigned long long key = s_mkey;
          res[w] = make_int4((int)(key >> 40), w + (int)((key >> 32) & 0xFF),
                             (int)(key & 0xFFFFFFFFull), 1);
        } else {
          res[w] = make_int4(s_len, -1, -1, fin);
        }
      }
      break;
    }
    __syncthreads();  // s_r / s_lv are rewritten by the next walk
  }
  if (pf == 0x7fffffff && tid == 1 && nw < 0) res[0].x = pf;  // never true: keeps the prefetch
}

// Follow the merges from walker 0 and copy the true rows into C.  Every block
// plans the chain from the walkers' results in LDS (a few hops) and copies a
// grid-stride share of the rows; block 0 writes the round state.
// res[w] = {a, t, b, 1}: walker w's row a equals walker t's row b;
//          {len, -1, -1, 2}: walker w reached the end, rows 0..len-1;
//          {len, -1, -1, 3}: history full, rows 0..len-1 (the chain ends there).
// rstate[0] = rounds (complete chain), rstate[1] = 1 if C overflows;
// *resume = round of the last true row when the sequential walk must go on, else -1.
__global__ void __launch_bounds__(256) k_walk_join(Tables t, const uint64_t* H, const int32_t* hn,
                                                   const int4* res, int nw, int Hcap,
                                                   int32_t* rstate, int32_t* resume) {
  constexpr int MAXSEG = 128, MAXW = 64;
  __shared__ int s_w[MAXSEG], s_e0[MAXSEG], s_g[MAXSEG], s_n[MAXSEG];
  __shared__ int4 s_res[MAXW];
  __shared__ int s_hn[MAXW];
  __shared__ int s_ns, s_ok;
  const int N = t.N;
  // one parallel load of every walker's result: the chain below is a few LDS hops
  for (int w = threadIdx.x; w < nw && w < MAXW; w += blockDim.x) {
    s_res[w] = res[w];
    s_hn[w] = hn[w];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int wc = 0, e = 0, g = 0, ns = 0, rs_out = -1, R = -1;
    auto emit = [&](int wv, int e0, int e1) {
      if (e1 > e0 && ns < MAXSEG) {
        s_w[ns] = wv;
        s_e0[ns] = e0;
        s_g[ns] = g;
        s_n[ns] = e1 - e0;
        ns++;
        g += e1 - e0;
      }
    };
    for (int it = 0; it <= nw; it++) {
      const int4 rs = s_res[wc];
      if (rs.w == 1) {
        const int a = rs.x, tw = rs.y, b = rs.z;
        int ne;
        if (e <= a) {
          emit(wc, e, a);
          ne = b;
        } else {
          ne = b + (e - a);
        }
        if (ne < s_hn[tw]) {
          wc = tw;
          e = ne;
          continue;
        }
        // the merged row is not published in walker tw: go on sequentially from
        // the true row we stand on
        const int cur = e <= a ? a : e;
        emit(wc, cur, cur + 1);
        rs_out = g - 1;
        break;
      }
      emit(wc, e, rs.x);
      if (rs.w == 2) R = g;
      else rs_out = g - 1;
      break;
    }
    const bool over = g + 1 >= t.Rcap || ns >= MAXSEG;
    if (blockIdx.x == 0) {
      if (over) rstate[1] = 1;
      else if (R >= 0) rstate[0] = R;
      *resume = over ? -1 : rs_out;
    }
    s_ns = ns;
    s_ok = !over;
  }
  __syncthreads();
  if (!s_ok) return;
  // flattened over (row, column): every thread's copies are independent
  const int gt = blockIdx.x * blockDim.x + threadIdx.x, gs = gridDim.x * blockDim.x;
  const int ns = s_ns;
  const int rows = ns > 0 ? s_g[ns - 1] + s_n[ns - 1] : 0;
  for (int i = gt; i < rows * N; i += gs) {
    const int q = i / N, c = i - q * N;
    int sg = 0;
    while (sg + 1 < ns && s_g[sg + 1] <= q) sg++;
    t.C[i] = (int32_t)(uint32_t)H[((size_t)s_w[sg] * Hcap + s_e0[sg] + (q - s_g[sg])) * N + c];
  }
}

}  // namespace hge
