/*
 * synth.c — synthetic fetch slices for tests and bench.py (BASELINE.json configs).
 *
 * Batches are built like the reference producer / BatchProducer
 * (crates/fluvio-protocol/src/fixture.rs:42-54, crates/fluvio/src/producer/config.rs:20):
 * magic 2, producer_epoch -1, offset_delta = index, key None, Compression::None,
 * a batch closes before its record section would exceed 16384 bytes.  Each batch
 * is encoded exactly as Batch::encode writes it (batch.rs:398-430), CRC32C included.
 *
 *   kind 1 (C1): 256-byte printable-ASCII values, ~50 % with an SSN token ddd-dd-dddd
 *   kind 2 (C2): ~1 KB JSON log records {"level":..,"message":..,...}; ~50 % of the
 *                messages contain the word "timeout"
 *   kind 3     : decimal i32 values in [-1000, 1000] (aggregate-sum / filter_map inputs)
 *   kind 4     : mixed short values incl. invalid UTF-8, empty values and keys (edge cases)
 *   kind 5 (C4): JSON arrays of 1-16 elements, each an integer or a short ASCII string,
 *                no whitespace (array_map_json_array input)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t rs;
static uint64_t rnd(void) {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return rs;
}
static uint32_t rnd_n(uint32_t n) { return (uint32_t)(rnd() % n); }

static uint32_t crc_tab[8][256];
static int crc_ready;
static void crc_init(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    crc_tab[0][i] = c;
  }
  for (int t = 1; t < 8; t++)
    for (uint32_t i = 0; i < 256; i++) crc_tab[t][i] = (crc_tab[t - 1][i] >> 8) ^ crc_tab[0][crc_tab[t - 1][i] & 0xff];
  crc_ready = 1;
}
static uint32_t crc32c(const uint8_t *p, size_t n) {
  if (!crc_ready) crc_init();
  uint32_t c = 0xFFFFFFFFu;
  while (n >= 8) {
    uint32_t lo = (p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24)) ^ c;
    uint32_t hi = p[4] | (p[5] << 8) | (p[6] << 16) | ((uint32_t)p[7] << 24);
    c = crc_tab[7][lo & 0xff] ^ crc_tab[6][(lo >> 8) & 0xff] ^ crc_tab[5][(lo >> 16) & 0xff] ^ crc_tab[4][lo >> 24] ^
        crc_tab[3][hi & 0xff] ^ crc_tab[2][(hi >> 8) & 0xff] ^ crc_tab[1][(hi >> 16) & 0xff] ^ crc_tab[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = crc_tab[0][(c ^ *p++) & 0xff] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

static size_t venc(int64_t num, uint8_t *o) {
  int64_t v = (int64_t)(((uint64_t)num << 1) ^ (uint64_t)(num >> 31));
  size_t k = 0;
  while (v & (int64_t)0xffffff80) {
    o[k++] = (uint8_t)((v & 0x7f) | 0x80);
    v >>= 7;
  }
  o[k++] = (uint8_t)v;
  return k;
}
static size_t vsz(int64_t num) {
  uint8_t t[16];
  return venc(num, t);
}
static void be(uint8_t *p, uint64_t v, int n) {
  for (int i = 0; i < n; i++) p[i] = (uint8_t)(v >> (8 * (n - 1 - i)));
}

static const char *WORDS[] = {"request", "served", "client", "connection", "database", "latency", "cache",
                              "miss",    "retry",  "worker", "shutdown",   "started",  "user",    "session",
                              "token",   "expired", "queue", "backlog",    "partition", "leader", "replica",
                              "commit",  "offset", "segment", "rolled",    "index",    "compaction", "stream"};
#define NWORDS (sizeof WORDS / sizeof WORDS[0])

/* value generators: write into v, return length */
static size_t gen_c1(uint8_t *v) {
  const size_t n = 256;
  for (size_t i = 0; i < n; i++) v[i] = (uint8_t)(32 + rnd_n(95));
  if (rnd() & 1) {
    size_t p = rnd_n((uint32_t)(n - 11));
    for (int k = 0; k < 11; k++) v[p + k] = (uint8_t)('0' + rnd_n(10));
    v[p + 3] = '-';
    v[p + 6] = '-';
  }
  return n;
}
static size_t put(char *o, size_t k, const char *s) {
  size_t n = strlen(s);
  memcpy(o + k, s, n);
  return k + n;
}
static size_t put_u(char *o, size_t k, uint32_t v, int width) {
  char t[12];
  int n = 0;
  do {
    t[n++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  while (n < width) t[n++] = '0';
  while (n) o[k++] = t[--n];
  return k;
}
static size_t gen_c2(uint8_t *v) {
  static const char *LV[] = {"debug", "info", "warn", "error"};
  static size_t wl[NWORDS];
  if (!wl[0])
    for (size_t i = 0; i < NWORDS; i++) wl[i] = strlen(WORDS[i]);
  char *o = (char *)v;
  size_t k = 0;
  k = put(o, k, "{\"level\":\"");
  k = put(o, k, LV[rnd_n(4)]);
  k = put(o, k, "\",\"message\":\"");
  const int timeout = (int)(rnd() & 1);
  const size_t target = 1024 - 80;
  int placed = 0;
  while (k < target) {
    if (timeout && !placed && k > 100 && rnd_n(8) == 0) {
      k = put(o, k, "timeout ");
      placed = 1;
      continue;
    }
    const uint32_t w = rnd_n(NWORDS);
    memcpy(o + k, WORDS[w], wl[w]);
    k += wl[w];
    o[k++] = ' ';
  }
  if (timeout && !placed) k = put(o, k, "timeout ");
  k = put(o, k, "\",\"service\":\"svc-");
  k = put_u(o, k, rnd_n(100), 2);
  k = put(o, k, "\",\"host\":\"h-");
  k = put_u(o, k, rnd_n(10000), 4);
  k = put(o, k, "\",\"ts\":");
  k = put_u(o, k, rnd_n(1000000000), 1);
  o[k++] = '}';
  return k;
}
/* ground truth of the last generated slice for the bench's state checks:
 * kind 3 = the i64 sum of the committed records' integers; synth_keyed = per
 * key index, the sum of its committed values (synth_key_sums, when set) */
static int64_t g_vsum;
static int g_last_c3;
static uint64_t *g_ksum;
int64_t synth_last_sum(void) { return g_vsum; }
void synth_key_sums(uint64_t *sums) { g_ksum = sums; }

static size_t gen_c3(uint8_t *v) {
  int x = (int)rnd_n(2001) - 1000;
  g_last_c3 = x;
  return (size_t)sprintf((char *)v, "%d", x);
}
static size_t gen_c4(uint8_t *v, int *has_key, uint8_t *key, size_t *klen) {
  uint32_t t = rnd_n(16);
  size_t n = 0;
  *has_key = rnd_n(4) == 0;
  *klen = 0;
  if (*has_key) {
    *klen = rnd_n(6);
    for (size_t i = 0; i < *klen; i++) key[i] = (uint8_t)('a' + rnd_n(26));
  }
  if (t == 0) return 0;                                   /* empty value */
  if (t == 1) {                                           /* invalid UTF-8 somewhere */
    n = 1 + rnd_n(20);
    for (size_t i = 0; i < n; i++) v[i] = (uint8_t)('a' + rnd_n(26));
    v[rnd_n((uint32_t)n)] = (uint8_t)(0x80 + rnd_n(0x80));
    return n;
  }
  if (t == 2) {                                           /* valid multi-byte UTF-8 */
    const char *s[] = {"caf\xc3\xa9 a", "\xe2\x82\xac" "12", "\xf0\x9f\x98\x80 ab", "\xd9\xa3\xd9\xa1"};
    const char *c = s[rnd_n(4)];
    n = strlen(c);
    memcpy(v, c, n);
    return n;
  }
  if (t <= 7) return (size_t)sprintf((char *)v, "%d", (int)rnd_n(200) - 100); /* ints */
  if (t == 8) return (size_t)sprintf((char *)v, " %d\t", (int)rnd_n(2000)); /* padded ints */
  n = 1 + rnd_n(40);
  for (size_t i = 0; i < n; i++) v[i] = (uint8_t)(32 + rnd_n(95));
  return n;
}

static size_t gen_c5(uint8_t *v) {
  char *o = (char *)v;
  size_t k = 0;
  const uint32_t ne = 1 + rnd_n(16);
  o[k++] = '[';
  for (uint32_t e = 0; e < ne; e++) {
    if (e) o[k++] = ',';
    if (rnd() & 1) {
      k += (size_t)sprintf(o + k, "%d", (int)rnd_n(200001) - 100000);
    } else {
      const uint32_t n = 1 + rnd_n(8);
      o[k++] = '"';
      for (uint32_t i = 0; i < n; i++) o[k++] = (char)('a' + rnd_n(26));
      o[k++] = '"';
    }
  }
  o[k++] = ']';
  return k;
}

/* Generate `nrec` records of `kind` into out (capacity cap) starting at base offset
 * `base`.  Returns bytes written, or 0 if cap is too small. */
size_t synth_slice(int kind, uint64_t nrec, uint64_t seed, int64_t base, uint8_t *out, size_t cap,
                   uint32_t max_section) {
  rs = seed * 0x9E3779B97F4A7C15ull + 0x1234567ull;
  if (!rs) rs = 1;
  g_vsum = 0;
  if (!max_section) max_section = 16384;
  size_t pos = 0;
  uint64_t done = 0;
  static uint8_t val[4096], key[64], rec[8192];
  while (done < nrec) {
    /* batch */
    if (pos + 61 > cap) return 0;
    uint8_t *bh = out + pos;
    size_t q = pos + 61;
    uint32_t cnt = 0;
    size_t sec = 4;
    for (;;) {
      if (done + cnt >= nrec) break;
      /* generate the next record into rec */
      int hk = 0;
      size_t kl = 0, vl;
      uint64_t save = rs;
      switch (kind) {
        case 1: vl = gen_c1(val); break;
        case 2: vl = gen_c2(val); break;
        case 3: vl = gen_c3(val); break;
        case 5: vl = gen_c5(val); break;
        default: vl = gen_c4(val, &hk, key, &kl); break;
      }
      size_t inner = 1 + vsz(0) + vsz((int64_t)cnt) + 1 + (hk ? vsz((int64_t)kl) + kl : 0) + vsz((int64_t)vl) + vl + 1;
      size_t rl = vsz((int64_t)inner) + inner;
      if (cnt > 0 && sec + rl > max_section) {
        rs = save; /* regenerate this record in the next batch */
        break;
      }
      size_t w = venc((int64_t)inner, rec);
      rec[w++] = 0;               /* attributes */
      w += venc(0, rec + w);      /* timestamp_delta */
      w += venc((int64_t)cnt, rec + w); /* offset_delta */
      rec[w++] = hk ? 1 : 0;
      if (hk) {
        w += venc((int64_t)kl, rec + w);
        memcpy(rec + w, key, kl);
        w += kl;
      }
      w += venc((int64_t)vl, rec + w);
      memcpy(rec + w, val, vl);
      w += vl;
      rec[w++] = 0; /* headers */
      if (q + w > cap) return 0;
      memcpy(out + q, rec, w);
      q += w;
      sec += w;
      if (kind == 3) g_vsum += g_last_c3;
      cnt++;
    }
    const int64_t first_ts = 1700000000000LL + (int64_t)(done / 64);
    be(bh + 0, (uint64_t)(base + (int64_t)done), 8);
    be(bh + 8, (uint32_t)(45 + sec), 4);
    be(bh + 12, 0, 4);        /* partition_leader_epoch */
    bh[16] = 2;               /* magic */
    be(bh + 21, 0, 2);        /* attributes */
    be(bh + 23, cnt - 1, 4);  /* last_offset_delta */
    be(bh + 27, (uint64_t)first_ts, 8);
    be(bh + 35, (uint64_t)first_ts, 8);
    be(bh + 43, 0, 8);        /* producer_id */
    be(bh + 51, (uint16_t)-1, 2);
    be(bh + 53, (uint32_t)-1, 4);
    be(bh + 57, cnt, 4);
    be(bh + 17, crc32c(bh + 21, q - (pos + 21)), 4);
    pos = q;
    done += cnt;
  }
  return pos;
}


/* C5 keyed (aggregate-json input): records `{"<key>":n}` (n in 1..100) whose
 * record key is the same <key>, picked uniformly from the caller's key list
 * (the keys SipHash routes to this partition).  keys = concatenated key bytes,
 * koff[k] .. koff[k + 1] = key k.  ~16 KiB record sections. */
size_t synth_keyed(const uint8_t *keys, const uint32_t *koff, uint32_t nkeys, uint64_t nrec, uint64_t seed,
                   int64_t base, uint8_t *out, size_t cap) {
  rs = seed * 0x9E3779B97F4A7C15ull + 0x7654321ull;
  if (!rs) rs = 1;
  size_t pos = 0;
  uint64_t done = 0;
  static uint8_t val[256], rec[512];
  while (done < nrec) {
    if (pos + 61 > cap) return 0;
    uint8_t *bh = out + pos;
    size_t q = pos + 61;
    uint32_t cnt = 0;
    size_t sec = 4;
    while (done + cnt < nrec) {
      const uint32_t k = rnd_n(nkeys);
      const uint8_t *kp = keys + koff[k];
      const size_t kl = koff[k + 1] - koff[k];
      if (kl > 64) return 0;
      size_t vl = 0;
      val[vl++] = '{';
      val[vl++] = '"';
      memcpy(val + vl, kp, kl);
      vl += kl;
      const uint32_t nv = 1 + rnd_n(100);
      vl += (size_t)sprintf((char *)val + vl, "\":%u}", nv);
      size_t inner = 1 + vsz(0) + vsz((int64_t)cnt) + 1 + vsz((int64_t)kl) + kl + vsz((int64_t)vl) + vl + 1;
      size_t rl = vsz((int64_t)inner) + inner;
      if (cnt > 0 && sec + rl > 16384) break;
      size_t w = venc((int64_t)inner, rec);
      rec[w++] = 0;
      w += venc(0, rec + w);
      w += venc((int64_t)cnt, rec + w);
      rec[w++] = 1;
      w += venc((int64_t)kl, rec + w);
      memcpy(rec + w, kp, kl);
      w += kl;
      w += venc((int64_t)vl, rec + w);
      memcpy(rec + w, val, vl);
      w += vl;
      rec[w++] = 0;
      if (q + w > cap) return 0;
      memcpy(out + q, rec, w);
      q += w;
      sec += w;
      if (g_ksum) g_ksum[k] += nv;
      cnt++;
    }
    const int64_t first_ts = 1700000000000LL + (int64_t)(done / 64);
    be(bh + 0, (uint64_t)(base + (int64_t)done), 8);
    be(bh + 8, (uint32_t)(45 + sec), 4);
    be(bh + 12, 0, 4);
    bh[16] = 2;
    be(bh + 21, 0, 2);
    be(bh + 23, cnt - 1, 4);
    be(bh + 27, (uint64_t)first_ts, 8);
    be(bh + 35, (uint64_t)first_ts, 8);
    be(bh + 43, 0, 8);
    be(bh + 51, (uint16_t)-1, 2);
    be(bh + 53, (uint32_t)-1, 4);
    be(bh + 57, cnt, 4);
    be(bh + 17, crc32c(bh + 21, q - (pos + 21)), 4);
    pos = q;
    done += cnt;
  }
  return pos;
}
