/*
 * ORACLE (test infrastructure only) — C restatement of the reference's hot path
 * over packed arrays.  Never linked into the product; loaded by tests/ and by
 * bench.py's cpu_baseline leg only.
 *
 *   classify  — mapper.py:159-189: candidate list per (acl, protocol) built as
 *               mapper.py:159-166 does (passed in, see oracle/coracle.py), scanned
 *               in order with FirewallRule.__contains__ (firewallrule.py:128-174):
 *               action equal (a logged connection is always permit, mapper.py:134),
 *               protocol 'ip' or equal, IPy containment of src and dst
 *               (ip >= net && ip < net + len), port-list membership unless [-1].
 *   reduce    — connlist-reducer.py:62-176 replayed per rule over its lines in
 *               sort order (the order key): hits for -6-302013/-6-302015 lines,
 *               then while len(conns) < cap the BUILT-regex lines insert/update
 *               (count, min ts, max ts) in first-seen order.
 *
 * Unlike the GPU (two passes + radix select of the cap threshold), this walks
 * the lines of each rule sequentially exactly like the reducer's loop.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint64_t key_hi; /* pspell << 48 | to_port << 32 | for_ip */
  uint32_t to_ip;
  uint32_t count, first, last;
  uint64_t first_order;
  int used;
} conn_t;

static int port_in(const int32_t *list, uint32_t len, uint32_t p) {
  for (uint32_t i = 0; i < len; ++i)
    if (list[i] == (int32_t)p) return 1;
  return 0;
}

/* rule tables (one entry per expanded rule, global index = gid) */
typedef struct {
  const uint8_t *action, *proto, *v4src, *v4dst;
  const uint32_t *src, *dst;
  const uint64_t *src_len, *dst_len; /* IPy len(): addresses in the network */
  const uint32_t *sp_off, *sp_len, *dp_off, *dp_len;
  const int32_t *ports;
  const uint64_t *src6, *dst6; /* IPv6 sides (v4* = 0): ip hi, ip lo, last hi, last lo per rule */
} rules_t;

static int contains(const rules_t *R, uint32_t g, uint32_t proto, uint32_t src, uint32_t dst, uint32_t sp,
                    uint32_t dp) {
  if (!R->action[g]) return 0;                                   /* firewallrule.py:146 */
  if (R->proto[g] != 0 && R->proto[g] != proto) return 0;       /* :150 (0 = 'ip')      */
  if (!R->v4src[g] || !R->v4dst[g]) return 0;                   /* IPy version mismatch  */
  if (!((uint64_t)src >= R->src[g] && (uint64_t)src < (uint64_t)R->src[g] + R->src_len[g])) return 0; /* :154 */
  if (!((uint64_t)dst >= R->dst[g] && (uint64_t)dst < (uint64_t)R->dst[g] + R->dst_len[g])) return 0; /* :158 */
  const int32_t *spl = R->ports + R->sp_off[g];
  if (!(R->sp_len[g] == 1 && spl[0] == -1) && !port_in(spl, R->sp_len[g], sp)) return 0; /* :162-165 */
  const int32_t *dpl = R->ports + R->dp_off[g];
  if (!(R->dp_len[g] == 1 && dpl[0] == -1) && !port_in(dpl, R->dp_len[g], dp)) return 0; /* :168-171 */
  return 1;
}

/* classify n tuples.  list_of[i] = candidate list id or -1 (line not classified);
 * cand[cand_off[l] .. cand_off[l+1]) = gids in scan order. */
void rsa_oracle_classify(uint64_t n, const int32_t *list_of, const uint32_t *proto_of, const uint32_t *src,
                         const uint32_t *dst, const uint32_t *sport, const uint32_t *dport, const uint32_t *cand_off,
                         const uint32_t *cand, const uint8_t *action, const uint8_t *proto, const uint8_t *v4src,
                         const uint8_t *v4dst, const uint32_t *rsrc, const uint32_t *rdst, const uint64_t *src_len,
                         const uint64_t *dst_len, const uint32_t *sp_off, const uint32_t *sp_len,
                         const uint32_t *dp_off, const uint32_t *dp_len, const int32_t *ports, int32_t *gid_out,
                         uint64_t *evals_out) {
  rules_t R = {action, proto, v4src, v4dst, rsrc, rdst, src_len, dst_len, sp_off, sp_len, dp_off, dp_len, ports,
               NULL, NULL};
  uint64_t evals = 0;
  /* lines are independent (one mapper call each): spread them over the host's
   * cores; each line is still the reference's sequential first-match scan */
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : evals)
  for (int64_t ii = 0; ii < (int64_t)n; ++ii) {
    const uint64_t i = (uint64_t)ii;
    gid_out[i] = -1;
    const int32_t l = list_of[i];
    if (l < 0) continue;
    for (uint32_t k = cand_off[l]; k < cand_off[l + 1]; ++k) {
      ++evals;
      if (contains(&R, cand[k], proto_of[i], src[i], dst[i], sport[i], dport[i])) {
        gid_out[i] = (int32_t)cand[k];
        break;
      }
    }
  }
  if (evals_out) *evals_out = evals;
}

static uint64_t hash2(uint64_t a, uint64_t b) {
  uint64_t x = a * 0x9e3779b97f4a7c15ull ^ (b + 0x632be59bd9b4e019ull);
  x ^= x >> 31;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 29;
  return x;
}

typedef struct {
  uint64_t order;
  uint64_t idx;
} ord_t;

static int cmp_ord(const void *a, const void *b) {
  const ord_t *x = (const ord_t *)a, *y = (const ord_t *)b;
  return x->order < y->order ? -1 : x->order > y->order ? 1 : (x->idx < y->idx ? -1 : x->idx > y->idx);
}

/* Reduce: per rule, replay the reducer loop over its lines in order-key order.
 * flags: bit1 HIT, bit2 BUILT, bit3 SWAP (as rsa_tuple.flags).
 * Outputs: matches[R], hits[R], n_conns[R] (len(conns) at the end),
 * and conn rows appended to out_* (capacity max_rows); returns rows written or
 * -1 if max_rows is too small.  Rows of one rule are contiguous, in first-seen order. */
int64_t rsa_oracle_reduce(uint64_t n, uint32_t n_rules, const int32_t *gid, const uint8_t *flags,
                          const uint8_t *pspell, const uint32_t *src, const uint32_t *dst, const uint32_t *sport,
                          const uint32_t *dport, const uint32_t *ts, const uint64_t *order, uint32_t cap,
                          uint64_t *matches, uint64_t *hits, uint32_t *n_conns, uint32_t *out_gid, uint32_t *out_for,
                          uint32_t *out_to, uint32_t *out_port, uint32_t *out_pspell, uint32_t *out_count,
                          uint32_t *out_first, uint32_t *out_last, uint64_t max_rows) {
  memset(matches, 0, sizeof(uint64_t) * n_rules);
  memset(hits, 0, sizeof(uint64_t) * n_rules);
  memset(n_conns, 0, sizeof(uint32_t) * n_rules);
  /* bucket line indices by gid */
  uint64_t *cnt = (uint64_t *)calloc((size_t)n_rules + 1, sizeof(uint64_t));
  for (uint64_t i = 0; i < n; ++i)
    if (gid[i] >= 0) cnt[gid[i] + 1]++;
  for (uint32_t g = 0; g < n_rules; ++g) cnt[g + 1] += cnt[g];
  uint64_t total = cnt[n_rules];
  ord_t *lines = (ord_t *)malloc(sizeof(ord_t) * (total ? total : 1));
  uint64_t *fill = (uint64_t *)malloc(sizeof(uint64_t) * ((size_t)n_rules + 1));
  memcpy(fill, cnt, sizeof(uint64_t) * ((size_t)n_rules + 1));
  for (uint64_t i = 0; i < n; ++i)
    if (gid[i] >= 0) {
      ord_t o = {order[i], i};
      lines[fill[gid[i]]++] = o;
    }
  uint64_t rows = 0;
  uint32_t tcap = 16;
  while (tcap < 2 * (cap + 1)) tcap <<= 1;
  conn_t *tab = (conn_t *)malloc(sizeof(conn_t) * tcap);
  uint32_t *ins = (uint32_t *)malloc(sizeof(uint32_t) * (cap + 1));
  int64_t rc = 0;
  for (uint32_t g = 0; g < n_rules; ++g) {
    const uint64_t b = cnt[g], e = cnt[g + 1];
    if (b == e) continue;
    qsort(lines + b, e - b, sizeof(ord_t), cmp_ord);
    memset(tab, 0, sizeof(conn_t) * tcap);
    uint32_t len = 0;
    for (uint64_t k = b; k < e; ++k) {
      const uint64_t i = lines[k].idx;
      matches[g]++;
      if (!(flags[i] & 2)) continue;          /* connlist-reducer.py:146 */
      hits[g]++;
      if (len >= cap) continue;               /* :151 */
      if (!(flags[i] & 4)) continue;          /* :152-153 BUILT regex */
      const int swap = flags[i] & 8;
      const uint32_t f = swap ? dst[i] : src[i];
      const uint32_t t = swap ? src[i] : dst[i];
      const uint32_t p = swap ? sport[i] : dport[i];
      const uint64_t khi = ((uint64_t)pspell[i] << 48) | ((uint64_t)p << 32) | f;
      uint64_t h = hash2(khi, t) & (tcap - 1);
      while (tab[h].used && !(tab[h].key_hi == khi && tab[h].to_ip == t)) h = (h + 1) & (tcap - 1);
      conn_t *c = &tab[h];
      if (!c->used) {                          /* :174-176 */
        c->used = 1;
        c->key_hi = khi;
        c->to_ip = t;
        c->count = 1;
        c->first = c->last = ts[i];
        c->first_order = order[i];
        ins[len++] = (uint32_t)h;
      } else {                                 /* :167-173 */
        c->count++;
        if (ts[i] < c->first) c->first = ts[i];
        if (ts[i] > c->last) c->last = ts[i];
      }
    }
    n_conns[g] = len;
    for (uint32_t j = 0; j < len; ++j) {
      if (rows >= max_rows) {
        rc = -1;
        goto done;
      }
      const conn_t *c = &tab[ins[j]];
      out_gid[rows] = g;
      out_for[rows] = (uint32_t)(c->key_hi & 0xFFFFFFFFu);
      out_port[rows] = (uint32_t)((c->key_hi >> 32) & 0xFFFFu);
      out_pspell[rows] = (uint32_t)(c->key_hi >> 48);
      out_to[rows] = c->to_ip;
      out_count[rows] = c->count;
      out_first[rows] = c->first;
      out_last[rows] = c->last;
      rows++;
    }
  }
  rc = (int64_t)rows;
done:
  free(cnt);
  free(lines);
  free(fill);
  free(tab);
  free(ins);
  return rc;
}

/* preprosess_access_lists.py:508-521 over rules [beg, end): cover[k] = the first
 * j in [beg, beg + k) with rule (beg + k) in rule j (FirewallRule.__contains__,
 * firewallrule.py:128-174, rule vs rule), or -1.  A plain double loop. */
typedef unsigned __int128 u128;
static u128 w128(const uint64_t *a, int k) { return ((u128)a[k] << 64) | a[k + 1]; }

/* IPv6 network b (rule i) inside network a (rule j): IPy's
 * b.ip >= a.ip and b's last address <= a's last address */
static int in6(const uint64_t *A, uint32_t j, uint32_t i) {
  return w128(A, 4 * i) >= w128(A, 4 * j) && w128(A, 4 * i + 2) <= w128(A, 4 * j + 2);
}

static int rule_in_rule(const rules_t *R, uint32_t j, uint32_t i) {
  if (R->action[j] != R->action[i]) return 0;                   /* :146 */
  if (R->proto[j] != 0 && R->proto[j] != R->proto[i]) return 0; /* :150 */
  /* IPy: an address of another version is never contained */
  if (R->v4src[j] != R->v4src[i] || R->v4dst[j] != R->v4dst[i]) return 0;
  if (R->v4src[i]) {
    if (!((uint64_t)R->src[i] >= R->src[j] && (uint64_t)R->src[i] + R->src_len[i] <= (uint64_t)R->src[j] + R->src_len[j]))
      return 0;                                                  /* :154 */
  } else if (!in6(R->src6, j, i)) {
    return 0;
  }
  if (R->v4dst[i]) {
    if (!((uint64_t)R->dst[i] >= R->dst[j] && (uint64_t)R->dst[i] + R->dst_len[i] <= (uint64_t)R->dst[j] + R->dst_len[j]))
      return 0;                                                  /* :158 */
  } else if (!in6(R->dst6, j, i)) {
    return 0;
  }
  const int32_t *sj = R->ports + R->sp_off[j], *si = R->ports + R->sp_off[i];
  if (!(R->sp_len[j] == 1 && sj[0] == -1))                      /* :162-165 */
    for (uint32_t q = 0; q < R->sp_len[i]; ++q)
      if (!port_in(sj, R->sp_len[j], (uint32_t)si[q])) return 0;
  const int32_t *dj = R->ports + R->dp_off[j], *di = R->ports + R->dp_off[i];
  if (!(R->dp_len[j] == 1 && dj[0] == -1))                      /* :168-171 */
    for (uint32_t q = 0; q < R->dp_len[i]; ++q)
      if (!port_in(dj, R->dp_len[j], (uint32_t)di[q])) return 0;
  return 1;
}

void rsa_oracle_shadow(uint32_t beg, uint32_t end, const uint8_t *action, const uint8_t *proto, const uint8_t *v4src,
                       const uint8_t *v4dst, const uint32_t *rsrc, const uint32_t *rdst, const uint64_t *src_len,
                       const uint64_t *dst_len, const uint32_t *sp_off, const uint32_t *sp_len, const uint32_t *dp_off,
                       const uint32_t *dp_len, const int32_t *ports, const uint64_t *src6, const uint64_t *dst6,
                       int32_t *cover) {
  rules_t R = {action, proto, v4src, v4dst, rsrc, rdst, src_len, dst_len, sp_off, sp_len, dp_off, dp_len, ports,
               src6, dst6};
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t k = 0; k < (int64_t)(end - beg); ++k) {
    const uint32_t i = beg + (uint32_t)k;
    cover[k] = -1;
    for (uint32_t j = beg; j < i; ++j)
      if (rule_in_rule(&R, j, i)) {
        cover[k] = (int32_t)(j - beg);
        break;
      }
  }
}
