/*
 * ratis_oracle.c -- CPU restatement of the reference's hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity oracle for libratis_hip.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker (or the timed CPU
 * baseline).  The product (ratis_amd/ + libratis_hip.so) never links or calls it.
 *
 * Every function restates one reference method, line by line, and cites it.  Reference paths
 * are relative to the OneSizeFitsQuorum/ratis tree:
 *   LSI = ratis-server/src/main/java/org/apache/ratis/server/impl/LeaderStateImpl.java
 *   RLB = ratis-server/src/main/java/org/apache/ratis/server/raftlog/RaftLogBase.java
 *   PJC = ratis-common/src/main/java/org/apache/ratis/util/PureJavaCrc32C.java
 *   OUT = ratis-server/.../raftlog/segmented/SegmentedRaftLogOutputStream.java
 *   RDR = ratis-server/.../raftlog/segmented/SegmentedRaftLogReader.java
 *   FMT = ratis-server/.../raftlog/segmented/SegmentedRaftLogFormat.java
 *
 * Pinning (see DESIGN.md "Oracle"):
 *   - CRC32C: the generated tables are compared word-for-word with the T[] text of PJC:167-688
 *     (tests/test_oracle.py, when /root/reference is present; a SHA-256 of the table is the
 *     committed fixture), plus RFC 3720 B.4 known answers.
 *   - Commit: the reference holds no golden vectors for getMajorityMin; the
 *     restatement is pinned by the majority-count rule of TestPeerConfiguration.java:45-70 and
 *     by hand-derived cases in tests/golden/commit_cases.json.
 *
 * Java semantics kept: all indices are signed 64-bit (Java long), `majority - min` wraps
 * (computed in uint64 to avoid C UB), sorting is ascending signed.
 */
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

#define ORC_API __attribute__((visibility("default")))

/* ===================================================================================== */
/* CRC32C -- PureJavaCrc32C                                                              */
/* ===================================================================================== */

static uint32_t T8[8][256];
static int T8_ready = 0;

/* Table generator: the reference's T[] comment names Hadoop's TestPureJavaCrc32$Table with
 * polynomial 82F63B78 (PJC:154-156).  T8_0 is the reflected byte-at-a-time table; T8_k[i] is
 * T8_{k-1}[i] advanced by one zero byte. */
static void orc_init_tables(void) {
    if (T8_ready) return;
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c >> 1) ^ ((c & 1u) ? 0x82F63B78u : 0u);
        T8[0][i] = c;
    }
    for (int t = 1; t < 8; t++)
        for (int i = 0; i < 256; i++)
            T8[t][i] = (T8[t - 1][i] >> 8) ^ T8[0][T8[t - 1][i] & 0xffu];
    T8_ready = 1;
}

/* Copies the 8x256 slicing table, laid out like PJC's T[] (T8_0 first). */
ORC_API void orc_crc32c_tables(uint32_t* out2048) {
    orc_init_tables();
    memcpy(out2048, T8, sizeof(T8));
}

/* PJC:49-51 reset(): crc = 0xffffffff.  State is the bit-flipped running value. */
ORC_API uint32_t orc_crc32c_reset(void) { return 0xffffffffu; }

/* PJC:43-46 getValue(): (~crc) & 0xffffffff. */
ORC_API uint32_t orc_crc32c_value(uint32_t state) { return ~state; }

/* PJC:54-91 update(byte[] b, int off, int len): slicing-by-8, Duff-style byte tail. */
ORC_API uint32_t orc_crc32c_update_array(uint32_t state, const uint8_t* b, size_t off, size_t len) {
    orc_init_tables();
    uint32_t localCrc = state;
    while (len > 7) {
        const uint32_t c0 = (b[off + 0] ^ localCrc) & 0xff;
        const uint32_t c1 = (b[off + 1] ^ (localCrc >>= 8)) & 0xff;
        const uint32_t c2 = (b[off + 2] ^ (localCrc >>= 8)) & 0xff;
        const uint32_t c3 = (b[off + 3] ^ (localCrc >>= 8)) & 0xff;
        localCrc = (T8[7][c0] ^ T8[6][c1]) ^ (T8[5][c2] ^ T8[4][c3]);
        const uint32_t c4 = b[off + 4];
        const uint32_t c5 = b[off + 5];
        const uint32_t c6 = b[off + 6];
        const uint32_t c7 = b[off + 7];
        localCrc ^= (T8[3][c4] ^ T8[2][c5]) ^ (T8[1][c6] ^ T8[0][c7]);
        off += 8;
        len -= 8;
    }
    while (len > 0) { /* PJC:77-87: case 7..1 each do one Sarwate step */
        localCrc = (localCrc >> 8) ^ T8[0][(localCrc ^ b[off++]) & 0xff];
        len--;
    }
    return localCrc;
}

/* PJC:93-147 update(ByteBuffer): little-endian 8-byte words, then 4/2/1-byte tails. */
ORC_API uint32_t orc_crc32c_update_bytebuffer(uint32_t state, const uint8_t* b, size_t off, size_t len) {
    orc_init_tables();
    uint32_t localCrc = state;
    while (len > 7) {
        uint64_t value = 0;
        for (int i = 7; i >= 0; i--) value = (value << 8) | b[off + (size_t)i];
        const uint32_t m = (uint32_t)value;
        const uint32_t n = (uint32_t)(value >> 32);
        const uint32_t c0 = ((m >> 0) ^ (localCrc >> 0)) & 0xff;
        const uint32_t c1 = ((m >> 8) ^ (localCrc >> 8)) & 0xff;
        const uint32_t c2 = ((m >> 16) ^ (localCrc >> 16)) & 0xff;
        const uint32_t c3 = ((m >> 24) ^ (localCrc >> 24)) & 0xff;
        const uint32_t c4 = (n >> 0) & 0xff;
        const uint32_t c5 = (n >> 8) & 0xff;
        const uint32_t c6 = (n >> 16) & 0xff;
        const uint32_t c7 = (n >> 24) & 0xff;
        localCrc = (T8[7][c0] ^ T8[6][c1]) ^ (T8[5][c2] ^ T8[4][c3]) ^
                   (T8[3][c4] ^ T8[2][c5]) ^ (T8[1][c6] ^ T8[0][c7]);
        off += 8;
        len -= 8;
    }
    if (len > 3) {
        const uint32_t n = (uint32_t)b[off] | ((uint32_t)b[off + 1] << 8) |
                           ((uint32_t)b[off + 2] << 16) | ((uint32_t)b[off + 3] << 24);
        for (int k = 0; k < 4; k++)
            localCrc = (localCrc >> 8) ^ T8[0][(localCrc ^ (n >> (8 * k))) & 0xff];
        off += 4;
        len -= 4;
    }
    if (len > 1) {
        const uint32_t n = (uint32_t)b[off] | ((uint32_t)b[off + 1] << 8);
        localCrc = (localCrc >> 8) ^ T8[0][(localCrc ^ (n >> 0)) & 0xff];
        localCrc = (localCrc >> 8) ^ T8[0][(localCrc ^ (n >> 8)) & 0xff];
        off += 2;
        len -= 2;
    }
    if (len > 0) localCrc = (localCrc >> 8) ^ T8[0][(localCrc ^ b[off]) & 0xff];
    return localCrc;
}

/* Convenience: value of a fresh PureJavaCrc32C after update(b, 0, len). */
ORC_API uint32_t orc_crc32c(const uint8_t* b, size_t len) {
    return orc_crc32c_value(orc_crc32c_update_array(orc_crc32c_reset(), b, 0, len));
}

/* Multi-threaded batch used only as the timed CPU baseline (bench.py cpu_baseline leg): one
 * fresh PureJavaCrc32C per frame over [off, off+len), compared against the stored big-endian
 * word that follows (RDR:327-336).  Returns the number of mismatches. */
ORC_API uint64_t orc_crc32c_frames(const uint8_t* buf, const uint64_t* off, const uint32_t* frame_len,
                                   uint64_t n, uint32_t* crc_out) {
    orc_init_tables();
    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t L = frame_len[i] - 4;
        const uint32_t c = orc_crc32c(buf + off[i], L);
        const uint8_t* s = buf + off[i] + L;
        const uint32_t stored = ((uint32_t)s[0] << 24) | ((uint32_t)s[1] << 16) | ((uint32_t)s[2] << 8) | s[3];
        if (crc_out) crc_out[i] = c;
        bad += (c != stored);
    }
    return bad;
}

/* ===================================================================================== */
/* Quorum commit -- LeaderStateImpl.getMajorityMin / updateCommit, RaftLogBase            */
/* ===================================================================================== */

/* MinMajorityMax (LSI:904-944). */
typedef struct { int64_t min, majority, max; } orc_mmm;

/* LSI:1076-1095 getSorted: followers in list order, then self (logIndex) last, then
 * Arrays.sort ascending.  For arrays shorter than 47 elements the JDK's DualPivotQuicksort.sort
 * (long[]) is a plain insertion sort (INSERTION_SORT_THRESHOLD), which is what runs here (n <= 15).
 * n == 0 throws IllegalArgumentException in Java; callers guard it. */
static int orc_get_sorted(const int64_t* follower_vals, const uint8_t* member, int nf, int include_self,
                          int64_t self_val, int64_t* out) {
    int n = 0;
    for (int i = 0; i < nf; i++) if (member[i]) out[n++] = follower_vals[i];
    if (include_self) out[n++] = self_val;
    for (int i = 1; i < n; i++) {
        const int64_t x = out[i];
        int j = i - 1;
        while (j >= 0 && out[j] > x) { out[j + 1] = out[j]; j--; }
        out[j + 1] = x;
    }
    return n;
}

/* LSI:926-935 valueOf(sorted, gapThreshold) with getMajority (LSI:937-939) and getMax
 * (LSI:941-943).  Java `majority - min` is long arithmetic: wraps. */
static orc_mmm orc_value_of(const int64_t* sorted, int n, int64_t gap) {
    orc_mmm r;
    int64_t majority = sorted[(n - 1) / 2];
    const int64_t min = sorted[0];
    const int64_t diff = (int64_t)((uint64_t)majority - (uint64_t)min);
    if (gap != -1 && diff > gap) majority = min;
    r.min = min;
    r.majority = majority;
    r.max = sorted[n - 1];
    return r;
}

/* LSI:915-920 combine: element-wise Math.min. */
static orc_mmm orc_combine(orc_mmm a, orc_mmm b) {
    orc_mmm r;
    r.min = a.min < b.min ? a.min : b.min;
    r.majority = a.majority < b.majority ? a.majority : b.majority;
    r.max = a.max < b.max ? a.max : b.max;
    return r;
}

/* LSI:956-984 getMajorityMin(followerIndex, logIndex, gapThreshold).
 *   follower_vals[nf]: the index column (matchIndex or commitIndex) of every follower slot.
 *   in_new[i] / in_old[i]: follower i is a voter of conf / oldConf with a FollowerInfo
 *   (LSI:291-293 filter(Objects::nonNull) over PeerConfiguration.streamPeerIds()).
 *   include_self = conf.containsInConf(selfId); include_self_old = conf.containsInOldConf(selfId).
 * Returns 1 and fills out[3] = {min, majority, max} for Optional.of, 0 for Optional.empty(). */
ORC_API int orc_get_majority_min(const int64_t* follower_vals, int nf, const uint8_t* in_new,
                                 const uint8_t* in_old, int include_self, int transitional,
                                 int include_self_old, int64_t self_val, int64_t gap, int64_t* out) {
    int64_t buf[64];
    if (nf > 63) return -1;
    int n_new = 0;
    for (int i = 0; i < nf; i++) n_new += in_new[i] != 0;
    if (n_new == 0 && !include_self) return 0;                                  /* LSI:964-966 */
    int n = orc_get_sorted(follower_vals, in_new, nf, include_self, self_val, buf);
    orc_mmm r = orc_value_of(buf, n, gap);                                       /* LSI:968-969 */
    if (transitional) {                                                          /* LSI:971-983 */
        int n_old = 0;
        for (int i = 0; i < nf; i++) n_old += in_old[i] != 0;
        if (n_old == 0 && !include_self_old) return 0;                          /* LSI:976-978 */
        n = orc_get_sorted(follower_vals, in_old, nf, include_self_old, self_val, buf);
        r = orc_combine(r, orc_value_of(buf, n, gap));
    }
    out[0] = r.min;
    out[1] = r.majority;
    out[2] = r.max;
    return 1;
}

/* Literal SegmentedRaftLogCache.getTermIndex(i).getTerm() over an explicit term array covering
 * log indices [log_start, log_start + n_terms); outside -> null (SegmentedRaftLogCache.java:550-557). */
static int orc_term_at(int64_t idx, int64_t log_start, const int64_t* terms, int64_t n_terms, int64_t* term) {
    if (idx < log_start || idx >= log_start + n_terms) return 0;
    *term = terms[idx - log_start];
    return 1;
}

/* RLB:121-142 updateCommitIndex(majorityIndex, currentTerm, isLeader=true), with the literal
 * term lookup.  Returns 1 iff the commit index was stored. */
ORC_API int orc_update_commit_index(int64_t* commit_index, int64_t majority, int64_t flush_index,
                                    int64_t current_term, int64_t log_start, const int64_t* terms,
                                    int64_t n_terms) {
    const int64_t oldCommittedIndex = *commit_index;
    const int64_t newCommitIndex = majority < flush_index ? majority : flush_index;   /* RLB:125 */
    if (oldCommittedIndex < newCommitIndex) {
        int64_t t;
        if (orc_term_at(newCommitIndex, log_start, terms, n_terms, &t) && t == current_term) {
            *commit_index = newCommitIndex;  /* RaftLogIndex.updateIncreasingly */
            return 1;
        }
    }
    return 0;
}

/* LSI:1015-1026 updateCommit(majority, min) followed by RLB:121-142.  `watch_all` receives
 * min (watchRequests.update(ALL, min), LSI:1025).  Returns 1 iff committed. */
ORC_API int orc_update_commit(int64_t* commit_index, int64_t majority, int64_t min, int64_t flush_index,
                              int64_t current_term, int64_t log_start, const int64_t* terms, int64_t n_terms,
                              int64_t* watch_all) {
    int advanced = 0;
    const int64_t oldLastCommitted = *commit_index;
    if (majority > oldLastCommitted)                                                   /* LSI:1017 */
        advanced = orc_update_commit_index(commit_index, majority, flush_index, current_term,
                                           log_start, terms, n_terms);
    *watch_all = min;
    return advanced;
}

/* ------------------------------------------------------------------------------------- */
/* Batched SoA driver with the exact argument layout of libratis_hip's rh_commit_soa      */
/* (include/ratis_hip.h).  The per-group work is the literal restatement above; the term */
/* lookup uses a two-term synthetic log: entries in [log_start, term_start) carry term    */
/* current-1, entries in [term_start, flush] carry current (monotone terms, LSI:296-301). */
/* ------------------------------------------------------------------------------------- */

#define ORC_CONF_NEW_MASK(w)    ((w) & 0x3FFFu)
#define ORC_CONF_SELF(w)        (((w) >> 14) & 1u)
#define ORC_CONF_TRANSITIONAL(w) (((w) >> 15) & 1u)
#define ORC_CONF_OLD_MASK(w)    (((w) >> 16) & 0x3FFFu)
#define ORC_CONF_SELF_OLD(w)    (((w) >> 30) & 1u)
#define ORC_CONF_ACTIVE(w)      (((w) >> 31) & 1u)

/* mode 0 = COMMIT (updateCommit, LSI:946-950), mode 1 = WATCH (commitIndexChanged, LSI:612-622). */
ORC_API void orc_commit_soa(uint64_t n, uint32_t nf, int mode, int64_t gap,
                            const int64_t* follower_index, /* [nf][n] */
                            const int64_t* self_index,     /* [n] flush (COMMIT) or lastCommitted (WATCH) */
                            const int64_t* commit_in, const int64_t* term_start, const int64_t* log_start,
                            const uint32_t* conf, int64_t* commit_out, int64_t* min_out, int64_t* maj_out,
                            int64_t* max_out, uint64_t* valid_bits, uint64_t* advanced_bits) {
    const uint64_t nwords = (n + 63) / 64;
    if (valid_bits) memset(valid_bits, 0, nwords * 8);
    if (advanced_bits) memset(advanced_bits, 0, nwords * 8);
    for (uint64_t g = 0; g < n; g++) {
        const uint32_t w = conf[g];
        int64_t vals[16];
        uint8_t in_new[16], in_old[16];
        for (uint32_t i = 0; i < nf; i++) {
            vals[i] = follower_index[(uint64_t)i * n + g];
            in_new[i] = (ORC_CONF_NEW_MASK(w) >> i) & 1u;
            in_old[i] = (ORC_CONF_OLD_MASK(w) >> i) & 1u;
        }
        int64_t mmm[3];
        int valid = 0;
        /* ABI rule (not Java's): a word naming a follower slot >= nf is malformed for this tier
         * and yields no result -- never a majority over fewer voters (include/ratis_hip.h). */
        const uint32_t fm = (1u << nf) - 1u;
        const int fits = (ORC_CONF_NEW_MASK(w) & ~fm) == 0 && (ORC_CONF_OLD_MASK(w) & ~fm) == 0;
        if (ORC_CONF_ACTIVE(w) && fits)
            valid = orc_get_majority_min(vals, (int)nf, in_new, in_old, (int)ORC_CONF_SELF(w),
                                         (int)ORC_CONF_TRANSITIONAL(w), (int)ORC_CONF_SELF_OLD(w),
                                         self_index[g], mode == 0 ? gap : -1, mmm);
        int64_t c = commit_in[g];
        int adv = 0;
        if (valid && mode == 0) {
            /* updateCommit(majority, min) + updateCommitIndex over the synthetic two-term log
             * [log_start, flush]: termAt(i) == currentTerm <=> i >= term_start (monotone terms,
             * LSI:296-301).  orc_update_commit_index is the literal array lookup; tests check
             * the two agree on random logs. */
            const int64_t ls = log_start ? log_start[g] : INT64_MIN;
            const int64_t flush = self_index[g];
            const int64_t old = c;
            if (mmm[1] > old) {                                                   /* LSI:1017 */
                const int64_t nc = mmm[1] < flush ? mmm[1] : flush;               /* RLB:125 */
                if (old < nc && nc >= ls && nc <= flush && nc >= term_start[g]) { c = nc; adv = 1; }
            }
        }
        commit_out[g] = c;
        if (min_out) min_out[g] = valid ? mmm[0] : INT64_MIN;
        if (maj_out) maj_out[g] = valid ? mmm[1] : INT64_MIN;
        if (max_out) max_out[g] = valid ? mmm[2] : INT64_MIN;
        if (valid && valid_bits) valid_bits[g / 64] |= 1ull << (g % 64);
        if (adv && advanced_bits) advanced_bits[g / 64] |= 1ull << (g % 64);
    }
}

/* ===================================================================================== */
/* Leader lease -- LeaderStateImpl.hasLease (LSI:1229-1249), LeaderLease (LL:60-103),     */
/* RaftConfigurationImpl.hasMajority/isSingleton (RCI:265-298), PeerConfiguration (PC:    */
/* 152-169), Timestamp (TS:51-56, 87-112).  Literal list form; the GPU kernel works on    */
/* elapsed times and order statistics instead, and tests check the two agree.             */
/* ===================================================================================== */

/* Timestamp.compareTo (TS:109-112): sign of the wrapped difference. */
static int ts_compare(int64_t a, int64_t b) {
    const int64_t d = (int64_t)((uint64_t)a - (uint64_t)b);
    return d > 0 ? 1 : d == 0 ? 0 : -1;
}

/* Timestamp.elapsedTimeMs (TS:87-90) at a frozen System.nanoTime() == now. */
static int64_t ts_elapsed_ms(int64_t now, int64_t t) {
    const int64_t d = (int64_t)((uint64_t)now - (uint64_t)t);
    return d / 1000000;   /* Java long division truncates toward zero, as C does */
}

/* PeerConfiguration.hasMajority(Predicate, includeSelf) (PC:157-169); `peers` = the conf's
 * followers (size n) plus self when include_self. */
static int pc_has_majority(const uint8_t* active, int n, int include_self) {
    if (n == 0 && !include_self) return 1;
    int num = include_self ? 1 : 0;
    for (int i = 0; i < n; i++) num += active[i] ? 1 : 0;
    return num > (n + (include_self ? 1 : 0)) / 2;
}

/* LeaderLease.getMaxTimestampWithMajorityAck (LL:90-103): sort ascending, element size/2;
 * empty list -> currentTime(). */
static int64_t ll_max_ts_with_majority_ack(const int64_t* ts, int n, int64_t now) {
    if (n == 0) return now;
    int64_t a[32];
    for (int i = 0; i < n; i++) a[i] = ts[i];
    for (int i = 1; i < n; i++) {                 /* stable insertion sort by compareTo */
        const int64_t x = a[i];
        int j = i - 1;
        while (j >= 0 && ts_compare(a[j], x) > 0) { a[j + 1] = a[j]; j--; }
        a[j + 1] = x;
    }
    return a[n / 2];
}

/* LeaderStateImpl.hasLease() for one group, isRunning() && isReady() taken as true.
 * cur_ts / old_ts: lastRespondedAppendEntriesSendTime of the followers of the current / old
 * conf (self excluded, as FollowerInfoMap.getFollowerInfos yields them, LSI:291-293); old_ts is
 * used only when transitional.  Returns hasLease; *lease_out = the lease after any extension. */
ORC_API int orc_has_lease(int enabled, int64_t now, int64_t timeout_ms, const int64_t* cur_ts, int n_cur,
                          int self_in_cur, const int64_t* old_ts, int n_old, int self_in_old, int transitional,
                          int64_t lease_in, int64_t* lease_out, int* extended) {
    *lease_out = lease_in;
    *extended = 0;
    if (!enabled) return 0;                                                  /* LSI:1230-1232 */
    /* RCI:296-298 isSingleton: getCurrentPeers().size()==1 && getPreviousPeers().size()<=1 */
    const int singleton = (n_cur + self_in_cur) == 1 && (transitional ? n_old + self_in_old : 0) <= 1;
    /* checkLeaderLease (LSI:1246-1249) with LeaderLease.isValid (LL:60-62) */
    if (singleton || ts_elapsed_ms(now, lease_in) < timeout_ms) return 1;
    /* LeaderLease.extend (LL:68-85): active peers of current ++ old, by last response time */
    uint8_t act_cur[32], act_old[32];
    for (int i = 0; i < n_cur; i++) act_cur[i] = ts_elapsed_ms(now, cur_ts[i]) < timeout_ms;
    for (int i = 0; i < n_old; i++) act_old[i] = ts_elapsed_ms(now, old_ts[i]) < timeout_ms;
    /* conf.hasMajority(peers, selfId) (RCI:265-269 -> PC:152-155) */
    int maj = pc_has_majority(act_cur, n_cur, self_in_cur);
    if (transitional) maj = maj && pc_has_majority(act_old, n_old, self_in_old);
    if (maj) {
        const int64_t a = ll_max_ts_with_majority_ack(cur_ts, n_cur, now);
        const int64_t b = transitional ? ll_max_ts_with_majority_ack(old_ts, n_old, now) : now;  /* old==null */
        *lease_out = ts_compare(a, b) > 0 ? b : a;                           /* Timestamp.earliest */
        *extended = 1;
    }
    return singleton || ts_elapsed_ms(now, *lease_out) < timeout_ms;
}

/* Batched form over the SoA layout (same conf word as orc_commit_soa). */
ORC_API void orc_lease_soa(uint64_t n, uint32_t nf, int64_t now, int64_t timeout_ms,
                           const int64_t* follower_ts, /* [nf][n] */
                           const uint32_t* conf, const int64_t* lease_in, const uint64_t* enabled_bits,
                           int64_t* lease_out, uint64_t* has_lease_bits, uint64_t* extended_bits) {
    const uint64_t nwords = (n + 63) / 64;
    memset(has_lease_bits, 0, nwords * 8);
    if (extended_bits) memset(extended_bits, 0, nwords * 8);
    for (uint64_t g = 0; g < n; g++) {
        const uint32_t w = conf[g];
        const uint32_t fm = (1u << nf) - 1u;   /* same malformed-word rule as orc_commit_soa */
        const int fits = (ORC_CONF_NEW_MASK(w) & ~fm) == 0 && (ORC_CONF_OLD_MASK(w) & ~fm) == 0;
        if (!ORC_CONF_ACTIVE(w) || !fits) { lease_out[g] = lease_in[g]; continue; }
        int64_t cur[16], old[16];
        int nc = 0, no = 0;
        for (uint32_t i = 0; i < nf; i++) {
            const int64_t t = follower_ts[(uint64_t)i * n + g];
            if ((ORC_CONF_NEW_MASK(w) >> i) & 1u) cur[nc++] = t;
            if ((ORC_CONF_OLD_MASK(w) >> i) & 1u) old[no++] = t;
        }
        const int en = enabled_bits ? (int)((enabled_bits[g / 64] >> (g % 64)) & 1u) : 1;
        int ext = 0;
        int64_t lo = 0;
        const int has = orc_has_lease(en, now, timeout_ms, cur, nc, (int)ORC_CONF_SELF(w), old, no,
                                      (int)ORC_CONF_SELF_OLD(w), (int)ORC_CONF_TRANSITIONAL(w), lease_in[g], &lo, &ext);
        lease_out[g] = lo;
        if (has) has_lease_bits[g / 64] |= 1ull << (g % 64);
        if (ext && extended_bits) extended_bits[g / 64] |= 1ull << (g % 64);
    }
}

/* ===================================================================================== */
/* SegmentedRaftLog frames -- writer OUT:86-110, reader RDR:179-341, format FMT:30-80     */
/* ===================================================================================== */

/* CodedOutputStream.computeUInt32SizeNoTag (protobuf 3.25, shaded in ratis-thirdparty-misc 1.1.0). */
ORC_API int orc_varint32_size(uint32_t v) {
    if ((v & (~0u << 7)) == 0) return 1;
    if ((v & (~0u << 14)) == 0) return 2;
    if ((v & (~0u << 21)) == 0) return 3;
    if ((v & (~0u << 28)) == 0) return 4;
    return 5;
}

static int put_varint32(uint8_t* p, uint32_t v) {
    int i = 0;
    while (v >= 0x80) { p[i++] = (uint8_t)(v | 0x80); v >>= 7; }
    p[i++] = (uint8_t)v;
    return i;
}

/* OUT:86-110 write(entry): varint32(n) || proto(n) || BE u32 CRC32C(varint||proto). */
ORC_API uint32_t orc_frame_write(uint8_t* dst, const uint8_t* proto, uint32_t n) {
    int v = put_varint32(dst, n);
    memcpy(dst + v, proto, n);
    const uint32_t c = orc_crc32c(dst, (size_t)v + n);
    uint8_t* s = dst + v + n;
    s[0] = (uint8_t)(c >> 24); s[1] = (uint8_t)(c >> 16); s[2] = (uint8_t)(c >> 8); s[3] = (uint8_t)c;
    return (uint32_t)v + n + 4;
}

/* Decode status codes (mirroring the outcomes of RDR decodeEntry/readEntry). */
enum {
    ORC_OK = 0,           /* entry decoded, checksum matched                                   */
    ORC_END = 1,          /* EOF at an entry boundary, or terminator + all-zero padding (null)  */
    ORC_PARTIAL = 2,      /* EOFException mid-entry -> readEntry returns null (RDR:221-229)     */
    ORC_E_OVERSIZE = -1,  /* "Entry has size ... but MAX_OP_SIZE" (RDR:314-317)                */
    ORC_E_CHECKSUM = -2,  /* ChecksumException (RDR:330-336)                                   */
    ORC_E_PADDING = -3,   /* verifyTerminator: "Read extra bytes after the terminator" (:251-280)*/
    ORC_E_VARINT = -4,    /* malformed varint (CodedInputStream.readRawVarint32 throws)         */
    ORC_E_HEADER = -5     /* CorruptedFileException from verifyHeader (RDR:201-204)            */
};

/* RDR:291-341 decodeEntry at byte offset `pos` of a segment image (header already consumed).
 * Outputs: *entry_len = varint + proto length (the CRC-covered span), *crc_calc, *crc_stored,
 * *next = offset after the 4-byte checksum. */
ORC_API int orc_decode_entry(const uint8_t* seg, uint64_t len, uint64_t pos, uint32_t max_op,
                             uint32_t* entry_len, uint32_t* crc_calc, uint32_t* crc_stored, uint64_t* next) {
    if (pos >= len) return ORC_END;                                   /* RDR:299-302 EOF at boundary */
    const uint8_t first = seg[pos];
    if (first == 0) {                                                 /* FMT isTerminator; RDR:306-309 */
        for (uint64_t i = pos; i < len; i++) if (seg[i] != 0) { *next = i; return ORC_E_PADDING; }
        *next = len;
        return ORC_END;
    }
    /* CodedInputStream.readRawVarint32(firstByte, in) (protobuf 3.25): up to 5 bytes, then
     * discards up to 5 more continuation bytes of a 64-bit varint, else malformedVarint.  A
     * read() of -1 throws truncatedMessage -- an IOException that is NOT an EOFException, so
     * readEntry (RDR:215-241) rethrows it rather than returning null. */
    uint32_t result = 0;
    int shift = 0;
    uint64_t p = pos;
    int done = 0;
    for (int i = 0; i < 5; i++) {
        if (p >= len) return ORC_E_VARINT;
        const uint8_t b = seg[p++];
        result |= (uint32_t)(b & 0x7f) << shift;
        shift += 7;
        if ((b & 0x80) == 0) { done = 1; break; }
    }
    if (!done) {
        for (int i = 0; i < 5; i++) {
            if (p >= len) return ORC_E_VARINT;
            if ((seg[p++] & 0x80) == 0) { done = 1; break; }
        }
        if (!done) return ORC_E_VARINT;
    }
    const int32_t entryLength = (int32_t)result;
    if (entryLength > (int32_t)max_op) return ORC_E_OVERSIZE;        /* RDR:314-317 (signed compare) */
    if (entryLength < 0) return ORC_E_VARINT;                         /* negative size: parse fails */
    const uint32_t varintLength = (uint32_t)orc_varint32_size((uint32_t)entryLength);
    const uint64_t totalLength = (uint64_t)varintLength + (uint32_t)entryLength;
    /* checkBufferSize (RDR:343-352) asserts totalLength <= max: IllegalStateException, wrapped
     * into IOException by readEntry. */
    if (totalLength > max_op) return ORC_E_OVERSIZE;
    if (pos + totalLength > len) return ORC_PARTIAL;                  /* readFully EOFException */
    /* readInt: four read() calls, each LimitedInputStream.checkLimit(1) BEFORE the read
     * (RDR:66-82): past the limit -> IOException; EOF -> EOFException (partial). */
    for (uint32_t k = 1; k <= 4; k++) {
        if (totalLength + k > max_op) return ORC_E_OVERSIZE;
        if (pos + totalLength + k > len) return ORC_PARTIAL;
    }
    const uint32_t c = orc_crc32c(seg + pos, totalLength);           /* RDR:327-329 */
    const uint8_t* s = seg + pos + totalLength;
    const uint32_t stored = ((uint32_t)s[0] << 24) | ((uint32_t)s[1] << 16) | ((uint32_t)s[2] << 8) | s[3];
    *entry_len = (uint32_t)totalLength;
    *crc_calc = c;
    *crc_stored = stored;
    *next = pos + totalLength + 4;
    return c == stored ? ORC_OK : ORC_E_CHECKSUM;                    /* RDR:330-336 */
}

/* RDR:179-205 verifyHeader.  1 = matched, 0 = partially written (terminator fill), -5 = corrupt. */
ORC_API int orc_verify_header(const uint8_t* seg, uint64_t len) {
    static const char H[8] = {'R', 'a', 'f', 't', 'L', 'o', 'g', '1'};
    const uint64_t readLength = len < 8 ? len : 8;
    uint64_t match = 0;
    while (match < readLength && seg[match] == (uint8_t)H[match]) match++;
    if (readLength == 8 && match == 8) return 1;
    for (uint64_t i = match; i < readLength; i++) if (seg[i] != 0) return ORC_E_HEADER;
    return 0;
}

/* Whole-segment walk (LogSegment.readSegmentFile, LogSegment.java:166-196, via
 * SegmentedRaftLogInputStream.nextEntry): header, then decodeEntry until END/error.
 * Fills up to `cap` frame records; returns the number of OK frames, and *status the final
 * decode status (ORC_END on a clean segment). */
ORC_API uint64_t orc_segment_scan(const uint8_t* seg, uint64_t len, uint32_t max_op, uint64_t cap,
                                  uint64_t* frame_off, uint32_t* frame_len, uint32_t* frame_crc,
                                  int* status, uint64_t* stop_pos) {
    const int h = orc_verify_header(seg, len);
    if (h != 1) { *status = h == 0 ? ORC_END : ORC_E_HEADER; *stop_pos = 0; return 0; }
    uint64_t pos = 8, n = 0;
    for (;;) {
        uint32_t el = 0, cc = 0, cs = 0;
        uint64_t next = pos;
        const int st = orc_decode_entry(seg, len, pos, max_op, &el, &cc, &cs, &next);
        if (st != ORC_OK) { *status = st; *stop_pos = (st == ORC_E_PADDING) ? next : pos; return n; }
        if (n < cap) { frame_off[n] = pos; frame_len[n] = el + 4; frame_crc[n] = cc; }
        n++;
        pos = next;
    }
}
