/*
 * ratis_hip_jni.c -- the native half of org.apache.ratis.hip.RatisHip: every native method,
 * each a direct call into the C ABI of libratis_hip (include/ratis_hip.h).
 *
 * Build (in the ratis-hip module, with a JDK):
 *   cc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I<ratis_amd>/include \
 *      ratis_hip_jni.c -L<ratis_amd>/ratis_amd/lib -lratis_hip -o libratis_hip_jni.so
 * The ratis_amd repository has no JDK; tests/test_java_module.py compiles this file with
 * -fsyntax-only against a minimal declaration of the JNI functions it uses, so every call here
 * is checked against the ABI header's prototypes.
 *
 * Error mapping: RH_E_INVAL / RH_E_RANGE -> IllegalArgumentException, other negative statuses ->
 * IOException, message = rh_last_error() (thread-local in the library).  Every array / buffer size
 * is checked against the count the call will read or write before the library sees a pointer
 * (RatisHip.java checks the same on the Java side): a short array throws
 * IllegalArgumentException, a null one where the call needs it too.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ratis_hip.h"

#define CLS(name) Java_org_apache_ratis_hip_RatisHip_##name

static void throw_msg(JNIEnv* env, const char* cls, const char* msg) {
    jclass c = (*env)->FindClass(env, cls);
    if (c) (*env)->ThrowNew(env, c, msg);
}

static void throw_rh(JNIEnv* env, int rc) {
    throw_msg(env, (rc == RH_E_INVAL || rc == RH_E_RANGE) ? "java/lang/IllegalArgumentException" : "java/io/IOException",
              rh_last_error());
}

static void throw_arg(JNIEnv* env, const char* msg) { throw_msg(env, "java/lang/IllegalArgumentException", msg); }

static int check(JNIEnv* env, int rc) {
    if (rc < 0) throw_rh(env, rc);
    return rc;
}

/* 1 when `a` is non-null and holds at least `need` elements, else throws and returns 0. */
static int has_len(JNIEnv* env, jarray a, int64_t need, const char* what) {
    if (!a) {
        throw_arg(env, what);
        return 0;
    }
    if ((int64_t)(*env)->GetArrayLength(env, a) < need) {
        throw_arg(env, what);
        return 0;
    }
    return 1;
}

static rh_node* N(jlong h) { return (rh_node*)(intptr_t)h; }
static rh_ctx* C(jlong h) { return (rh_ctx*)(intptr_t)h; }

static rh_groups* shard_table(JNIEnv* env, jlong node, jint shard) {
    rh_groups* g = rh_node_groups(N(node), (int)shard);
    if (!g) throw_arg(env, "no such shard");
    return g;
}

JNIEXPORT jlong JNICALL CLS(nodeCreate0)(JNIEnv* env, jclass c, jint mask, jlong cap, jlong gap) {
    (void)c;
    rh_node* node = NULL;
    if (check(env, rh_node_create((uint32_t)mask, (uint64_t)cap, (int64_t)gap, &node)) < 0) return 0;
    return (jlong)(intptr_t)node;
}

JNIEXPORT void JNICALL CLS(nodeDestroy0)(JNIEnv* env, jclass c, jlong node) {
    (void)c;
    check(env, rh_node_destroy(N(node)));
}

JNIEXPORT jint JNICALL CLS(nodeShards0)(JNIEnv* env, jclass c, jlong node) {
    (void)c;
    return (jint)check(env, rh_node_shards(N(node)));
}

JNIEXPORT jint JNICALL CLS(shardOf0)(JNIEnv* env, jclass c, jlong msb, jlong lsb, jint shards) {
    (void)c;
    return (jint)check(env, rh_shard_of((uint64_t)msb, (uint64_t)lsb, (int)shards));
}

JNIEXPORT void JNICALL CLS(groupStart0)(JNIEnv* env, jclass c, jlong node, jint slot, jint conf, jlong flush,
                                        jlong commit, jlong term_start) {
    (void)c;
    check(env, rh_node_group_start(N(node), (uint32_t)slot, (uint32_t)conf, (int64_t)flush, (int64_t)commit,
                                   (int64_t)term_start));
}

JNIEXPORT void JNICALL CLS(groupReconf0)(JNIEnv* env, jclass c, jlong node, jint slot, jint conf, jbyteArray src) {
    (void)c;
    int8_t map[RH_MAX_FOLLOWERS];
    const int8_t* p = NULL;
    if (src) {
        if (!has_len(env, src, RH_MAX_FOLLOWERS, "src must hold 14 entries")) return;
        (*env)->GetByteArrayRegion(env, src, 0, (jsize)RH_MAX_FOLLOWERS, (jbyte*)map);
        p = map;
    }
    check(env, rh_node_group_reconf(N(node), (uint32_t)slot, (uint32_t)conf, p));
}

JNIEXPORT void JNICALL CLS(groupStop0)(JNIEnv* env, jclass c, jlong node, jint slot) {
    (void)c;
    check(env, rh_node_group_stop(N(node), (uint32_t)slot));
}

JNIEXPORT void JNICALL CLS(pushDeltas0)(JNIEnv* env, jclass c, jlong node, jobject direct, jint n) {
    (void)c;
    if (n < 0) {
        throw_arg(env, "negative delta count");
        return;
    }
    if (n == 0) return;
    const rh_delta* d = direct ? (const rh_delta*)(*env)->GetDirectBufferAddress(env, direct) : NULL;
    const jlong capb = direct ? (*env)->GetDirectBufferCapacity(env, direct) : -1;
    if (!d || capb < 0 || (int64_t)n > capb / (jlong)sizeof(rh_delta)) {
        throw_arg(env, "pushDeltas: not a direct buffer, or n deltas exceed its capacity");
        return;
    }
    check(env, rh_node_push_deltas(N(node), d, (size_t)n));
}

JNIEXPORT jobject JNICALL CLS(acquire0)(JNIEnv* env, jclass c, jlong node, jint shard) {
    (void)c;
    rh_groups* g = shard_table(env, node, shard);
    if (!g) return NULL;
    rh_delta* buf = NULL;
    size_t cap = 0;
    if (check(env, rh_deltas_acquire(g, &buf, &cap)) < 0) return NULL;
    return (*env)->NewDirectByteBuffer(env, buf, (jlong)(cap * sizeof(rh_delta)));
}

JNIEXPORT void JNICALL CLS(submit0)(JNIEnv* env, jclass c, jlong node, jint shard, jint n) {
    (void)c;
    if (n < 0 || (uint64_t)n > RH_DELTA_SLOT) {
        throw_arg(env, "submit: n outside [0, RH_DELTA_SLOT]");
        return;
    }
    rh_groups* g = shard_table(env, node, shard);
    if (g) check(env, rh_deltas_submit(g, (size_t)n));
}

/* Copies k events into (slot, value) arrays. */
static void put_events(JNIEnv* env, const rh_index_event* ev, jsize k, jintArray slot, jlongArray value, jint base) {
    if (k <= 0) return;
    jint* s = (*env)->GetPrimitiveArrayCritical(env, slot, NULL);
    jlong* v = s ? (*env)->GetPrimitiveArrayCritical(env, value, NULL) : NULL;
    if (s && v)
        for (jsize i = 0; i < k; ++i) {
            s[i] = (jint)ev[i].slot + base;
            v[i] = (jlong)ev[i].value;
        }
    if (v) (*env)->ReleasePrimitiveArrayCritical(env, value, v, 0);
    if (s) (*env)->ReleasePrimitiveArrayCritical(env, slot, s, 0);
}

JNIEXPORT jlong JNICALL CLS(commitBatch0)(JNIEnv* env, jclass c, jlong node, jintArray adv_slot,
                                          jlongArray adv_commit, jintArray wall_slot, jlongArray wall_min) {
    (void)c;
    if (!adv_slot) {
        throw_arg(env, "advSlot == null");
        return 0;
    }
    const jsize acap = (*env)->GetArrayLength(env, adv_slot);
    const jsize wcap = wall_slot ? (*env)->GetArrayLength(env, wall_slot) : 0;
    if (!has_len(env, adv_commit, acap, "advCommit shorter than advSlot")) return 0;
    if (wall_slot && !has_len(env, wall_min, wcap, "wallMin shorter than wallSlot")) return 0;
    rh_index_event* adv = (rh_index_event*)malloc(sizeof(rh_index_event) * (size_t)(acap ? acap : 1));
    rh_index_event* wall = (rh_index_event*)malloc(sizeof(rh_index_event) * (size_t)(wcap ? wcap : 1));
    uint64_t na = 0, nw = 0;
    const uint32_t flags = wall_slot ? RH_COMMIT_WATCH_ALL : 0u;   /* watch-ALL levels only when asked */
    int rc = (adv && wall) ? rh_node_commit_batch(N(node), flags, adv, (uint64_t)acap, &na, wall, (uint64_t)wcap, &nw)
                           : RH_E_NOMEM;
    if (rc >= 0) {
        put_events(env, adv, (jsize)(na < (uint64_t)acap ? na : (uint64_t)acap), adv_slot, adv_commit, 0);
        if (wall_slot) put_events(env, wall, (jsize)(nw < (uint64_t)wcap ? nw : (uint64_t)wcap), wall_slot, wall_min, 0);
    }
    free(adv);
    free(wall);
    if (check(env, rc) < 0) return 0;
    return (jlong)((na << 32) | (nw & 0xFFFFFFFFull));
}

JNIEXPORT jlong JNICALL CLS(commitAsync0)(JNIEnv* env, jclass c, jlong node, jint shard, jint flags) {
    (void)c;
    rh_groups* g = shard_table(env, node, shard);
    if (!g) return 0;
    uint64_t tk = 0;
    if (check(env, rh_commit_batch_async(g, (uint32_t)flags, &tk)) < 0) return 0;
    return (jlong)tk;
}

/* rh_tick_async: the shard's updateCommit and commitIndexChanged in one call (one launch when both
 * kinds' dirty rows are listed); collected with commitWait0 (the ticket) and watchWait0. */
JNIEXPORT jlong JNICALL CLS(tickAsync0)(JNIEnv* env, jclass c, jlong node, jint shard, jint flags) {
    (void)c;
    rh_groups* g = shard_table(env, node, shard);
    if (!g) return 0;
    uint64_t tk = 0;
    if (check(env, rh_tick_async(g, (uint32_t)flags, &tk)) < 0) return 0;
    return (jlong)tk;
}

/* The shard's events straight from the library's pinned result buffers into the caller's arrays
 * (slots within the shard); the arrays hold at least the shard capacity (checked in RatisHip). */
JNIEXPORT jlong JNICALL CLS(commitWait0)(JNIEnv* env, jclass c, jlong node, jint shard, jlong ticket,
                                         jintArray adv_slot, jlongArray adv_commit, jintArray wall_slot,
                                         jlongArray wall_min) {
    (void)c;
    rh_groups* g = shard_table(env, node, shard);
    if (!g) return 0;
    rh_commit_out o;
    memset(&o, 0, sizeof(o));
    if (check(env, rh_commit_batch_wait(g, (uint64_t)ticket, &o)) < 0) return 0;
    if (!has_len(env, adv_slot, (int64_t)o.n_advanced, "advSlot shorter than the events") ||
        !has_len(env, adv_commit, (int64_t)o.n_advanced, "advCommit shorter than the events") ||
        !has_len(env, wall_slot, (int64_t)o.n_watch_all, "wallSlot shorter than the events") ||
        !has_len(env, wall_min, (int64_t)o.n_watch_all, "wallMin shorter than the events"))
        return 0;
    put_events(env, o.advanced, (jsize)o.n_advanced, adv_slot, adv_commit, 0);
    put_events(env, o.watch_all, (jsize)o.n_watch_all, wall_slot, wall_min, 0);
    return (jlong)((o.n_advanced << 32) | (o.n_watch_all & 0xFFFFFFFFull));
}

/* Copies n level-change events into the caller's arrays (checked to hold them). */
static jint put_levels(JNIEnv* env, const rh_watch_event* ev, uint64_t n, jintArray slot, jlongArray mn,
                       jlongArray mj, jlongArray mx, jbooleanArray valid) {
    if (!has_len(env, slot, (int64_t)n, "slot shorter than the events") ||
        !has_len(env, mn, (int64_t)n, "min shorter than the events") ||
        !has_len(env, mj, (int64_t)n, "majority shorter than the events") ||
        !has_len(env, mx, (int64_t)n, "max shorter than the events") ||
        !has_len(env, valid, (int64_t)n, "valid shorter than the events"))
        return 0;
    if (n == 0) return 0;
    jint* s = (*env)->GetPrimitiveArrayCritical(env, slot, NULL);
    jlong* a = s ? (*env)->GetPrimitiveArrayCritical(env, mn, NULL) : NULL;
    jlong* b = a ? (*env)->GetPrimitiveArrayCritical(env, mj, NULL) : NULL;
    jlong* d = b ? (*env)->GetPrimitiveArrayCritical(env, mx, NULL) : NULL;
    jboolean* v = d ? (*env)->GetPrimitiveArrayCritical(env, valid, NULL) : NULL;
    if (v)
        for (uint64_t i = 0; i < n; ++i) {
            s[i] = (jint)ev[i].slot;
            a[i] = (jlong)ev[i].min;
            b[i] = (jlong)ev[i].majority;
            d[i] = (jlong)ev[i].max;
            v[i] = ev[i].valid ? JNI_TRUE : JNI_FALSE;
        }
    if (v) (*env)->ReleasePrimitiveArrayCritical(env, valid, v, 0);
    if (d) (*env)->ReleasePrimitiveArrayCritical(env, mx, d, 0);
    if (b) (*env)->ReleasePrimitiveArrayCritical(env, mj, b, 0);
    if (a) (*env)->ReleasePrimitiveArrayCritical(env, mn, a, 0);
    if (s) (*env)->ReleasePrimitiveArrayCritical(env, slot, s, 0);
    return (jint)n;
}

JNIEXPORT jint JNICALL CLS(watchLevels0)(JNIEnv* env, jclass c, jlong node, jint shard, jintArray slot,
                                         jlongArray mn, jlongArray mj, jlongArray mx, jbooleanArray valid) {
    (void)c;
    rh_groups* g = shard_table(env, node, shard);
    if (!g) return 0;
    const rh_watch_event* ev = NULL;
    uint64_t n = 0;
    if (check(env, rh_watch_levels(g, &ev, &n)) < 0) return 0;
    return put_levels(env, ev, n, slot, mn, mj, mx, valid);
}

JNIEXPORT void JNICALL CLS(watchAsync0)(JNIEnv* env, jclass c, jlong node, jint shard) {
    (void)c;
    rh_groups* g = shard_table(env, node, shard);
    if (g) check(env, rh_watch_levels_async(g));
}

JNIEXPORT jint JNICALL CLS(watchWait0)(JNIEnv* env, jclass c, jlong node, jint shard, jintArray slot,
                                       jlongArray mn, jlongArray mj, jlongArray mx, jbooleanArray valid) {
    (void)c;
    rh_groups* g = shard_table(env, node, shard);
    if (!g) return 0;
    const rh_watch_event* ev = NULL;
    uint64_t n = 0;
    if (check(env, rh_watch_levels_wait(g, &ev, &n)) < 0) return 0;
    return put_levels(env, ev, n, slot, mn, mj, mx, valid);
}

JNIEXPORT void JNICALL CLS(setEventSink0)(JNIEnv* env, jclass c, jlong node, jint shard, jint sink) {
    (void)c;
    rh_groups* g = shard_table(env, node, shard);
    if (g) check(env, rh_groups_set_event_sink(g, (int)sink));
}

JNIEXPORT void JNICALL CLS(leaseAsync0)(JNIEnv* env, jclass c, jlong node, jint shard, jlong now, jlong timeout_ms) {
    (void)c;
    rh_groups* g = shard_table(env, node, shard);
    if (g) check(env, rh_lease_batch_async(g, (int64_t)now, (int64_t)timeout_ms));
}

JNIEXPORT void JNICALL CLS(leaseWait0)(JNIEnv* env, jclass c, jlong node, jint shard, jlongArray bits) {
    (void)c;
    rh_groups* g = shard_table(env, node, shard);
    if (!g) return;
    const uint64_t* w = NULL;
    uint64_t words = 0;
    if (check(env, rh_lease_batch_wait(g, &w, &words)) < 0) return;
    if (!has_len(env, bits, (int64_t)words, "bits shorter than the shard bitmap")) return;
    (*env)->SetLongArrayRegion(env, bits, 0, (jsize)words, (const jlong*)w);
}

JNIEXPORT void JNICALL CLS(leaseStart0)(JNIEnv* env, jclass c, jlong node, jint slot, jlong now, jboolean enabled) {
    (void)c;
    check(env, rh_node_group_lease_start(N(node), (uint32_t)slot, (int64_t)now, enabled ? 1 : 0));
}

JNIEXPORT void JNICALL CLS(leaseBatch0)(JNIEnv* env, jclass c, jlong node, jlong now, jlong timeout_ms,
                                        jlongArray bits) {
    (void)c;
    if (!bits) {
        throw_arg(env, "bits == null");
        return;
    }
    const jsize n = (*env)->GetArrayLength(env, bits);
    jlong* b = (*env)->GetLongArrayElements(env, bits, NULL);
    if (!b) return;
    const int rc = rh_node_lease_batch(N(node), (int64_t)now, (int64_t)timeout_ms, (uint64_t*)b, (uint64_t)n);
    (*env)->ReleaseLongArrayElements(env, bits, b, rc < 0 ? JNI_ABORT : 0);
    check(env, rc);
}

JNIEXPORT void JNICALL CLS(leaseBatchShard0)(JNIEnv* env, jclass c, jlong node, jint shard, jlong now,
                                             jlong timeout_ms, jlongArray bits) {
    (void)c;
    rh_groups* g = shard_table(env, node, shard);
    if (!g) return;
    const uint64_t* w = NULL;
    uint64_t words = 0;
    if (check(env, rh_lease_batch(g, (int64_t)now, (int64_t)timeout_ms, &w, &words)) < 0) return;
    if (!has_len(env, bits, (int64_t)words, "bits shorter than the shard bitmap")) return;
    (*env)->SetLongArrayRegion(env, bits, 0, (jsize)words, (const jlong*)w);
}

JNIEXPORT jlong JNICALL CLS(verifyHost0)(JNIEnv* env, jclass c, jlong node, jint shard, jobject seg, jlong pos,
                                         jlong len, jlongArray off, jintArray flen, jint n, jintArray crc,
                                         jlongArray bad) {
    (void)c;
    rh_ctx* ctx = rh_node_ctx(N(node), (int)shard);
    const uint8_t* base = seg ? (const uint8_t*)(*env)->GetDirectBufferAddress(env, seg) : NULL;
    const jlong capb = seg ? (*env)->GetDirectBufferCapacity(env, seg) : -1;
    if (!ctx || !base || pos < 0 || len < 0 || capb < 0 || pos > capb || len > capb - pos || n < 0) {
        throw_arg(env, "verifyFrames: no such shard, not a direct buffer, or [position, limit) outside it");
        return 0;
    }
    if (!has_len(env, off, n, "frameOff shorter than n") || !has_len(env, flen, n, "frameLen shorter than n") ||
        (crc && !has_len(env, crc, n, "crcOut shorter than n")) ||
        (bad && !has_len(env, bad, ((int64_t)n + 63) / 64, "badBits shorter than ceil(n / 64)")))
        return 0;
    jlong* o = (*env)->GetLongArrayElements(env, off, NULL);
    jint* l = (*env)->GetIntArrayElements(env, flen, NULL);
    jint* cr = crc ? (*env)->GetIntArrayElements(env, crc, NULL) : NULL;
    jlong* b = bad ? (*env)->GetLongArrayElements(env, bad, NULL) : NULL;
    uint64_t nb = 0;
    const int rc = rh_crc32c_verify_host(ctx, base + pos, (uint64_t)len, (const uint64_t*)o, (const uint32_t*)l,
                                         (uint64_t)n, (uint32_t*)cr, (uint64_t*)b, &nb);
    if (b) (*env)->ReleaseLongArrayElements(env, bad, b, 0);
    if (cr) (*env)->ReleaseIntArrayElements(env, crc, cr, 0);
    (*env)->ReleaseIntArrayElements(env, flen, l, JNI_ABORT);
    (*env)->ReleaseLongArrayElements(env, off, o, JNI_ABORT);
    if (check(env, rc) < 0) return 0;
    return (jlong)nb;
}

/* ---- the log read path (HipLogReader) -------------------------------------------------------- */
JNIEXPORT jlong JNICALL CLS(ctxCreate0)(JNIEnv* env, jclass c, jint device) {
    (void)c;
    rh_ctx* ctx = NULL;
    if (check(env, rh_init((int)device, &ctx)) < 0) return 0;
    return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL CLS(ctxDestroy0)(JNIEnv* env, jclass c, jlong ctx) {
    (void)c;
    check(env, rh_shutdown(C(ctx)));
}

JNIEXPORT jlong JNICALL CLS(readSegments0)(JNIEnv* env, jclass c, jlong ctx, jobject image, jlong image_len,
                                           jlongArray seg_off, jlongArray seg_len, jint n_seg, jint max_op,
                                           jint cap_per_seg, jlongArray frame_off, jintArray frame_len,
                                           jintArray frame_crc, jintArray seg_ints, jlongArray seg_longs) {
    (void)c;
    const uint8_t* img = image ? (const uint8_t*)(*env)->GetDirectBufferAddress(env, image) : NULL;
    const jlong capb = image ? (*env)->GetDirectBufferCapacity(env, image) : -1;
    if (!img || image_len < 0 || capb < image_len || n_seg < 0 || max_op <= 0 || cap_per_seg <= 0) {
        throw_arg(env, "readSegments: not a direct buffer, imageLen beyond it, or a bad count");
        return 0;
    }
    if (!has_len(env, seg_off, n_seg, "segOff shorter than nSeg") || !has_len(env, seg_len, n_seg, "segLen shorter than nSeg") ||
        !has_len(env, seg_ints, 3 * (int64_t)n_seg, "segInts shorter than 3 * nSeg") ||
        !has_len(env, seg_longs, 2 * (int64_t)n_seg, "segLongs shorter than 2 * nSeg") || !frame_off || !frame_len) {
        if (!(*env)->ExceptionCheck(env)) throw_arg(env, "frameOff / frameLen == null");
        return 0;
    }
    const jsize fcap = (*env)->GetArrayLength(env, frame_off);
    if (!has_len(env, frame_len, fcap, "frameLen shorter than frameOff") ||
        (frame_crc && !has_len(env, frame_crc, fcap, "frameCrc shorter than frameOff")))
        return 0;
    rh_segment_result* res = (rh_segment_result*)calloc((size_t)(n_seg ? n_seg : 1), sizeof(rh_segment_result));
    if (!res) {
        throw_msg(env, "java/lang/OutOfMemoryError", "readSegments: results");
        return 0;
    }
    jlong* so = (*env)->GetLongArrayElements(env, seg_off, NULL);
    jlong* sl = (*env)->GetLongArrayElements(env, seg_len, NULL);
    jlong* fo = (*env)->GetLongArrayElements(env, frame_off, NULL);
    jint* fl = (*env)->GetIntArrayElements(env, frame_len, NULL);
    jint* fc = frame_crc ? (*env)->GetIntArrayElements(env, frame_crc, NULL) : NULL;
    uint64_t total = 0;
    const int rc = rh_segments_read_host(C(ctx), img, (uint64_t)image_len, (const uint64_t*)so, (const uint64_t*)sl,
                                         (uint64_t)n_seg, (uint32_t)max_op, (uint32_t)cap_per_seg, (uint64_t*)fo,
                                         (uint32_t*)fl, (uint32_t*)fc, (uint64_t)fcap, res, &total);
    if (fc) (*env)->ReleaseIntArrayElements(env, frame_crc, fc, rc < 0 ? JNI_ABORT : 0);
    (*env)->ReleaseIntArrayElements(env, frame_len, fl, rc < 0 ? JNI_ABORT : 0);
    (*env)->ReleaseLongArrayElements(env, frame_off, fo, rc < 0 ? JNI_ABORT : 0);
    (*env)->ReleaseLongArrayElements(env, seg_len, sl, JNI_ABORT);
    (*env)->ReleaseLongArrayElements(env, seg_off, so, JNI_ABORT);
    if (rc >= 0) {
        jint* si = (*env)->GetIntArrayElements(env, seg_ints, NULL);
        jlong* sg = (*env)->GetLongArrayElements(env, seg_longs, NULL);
        if (si && sg)
            for (jint s = 0; s < n_seg; ++s) {
                si[3 * s] = (jint)res[s].status;
                si[3 * s + 1] = (jint)res[s].n_ok;
                si[3 * s + 2] = (jint)res[s].n_frames;
                sg[2 * s] = (jlong)res[s].stop;
                sg[2 * s + 1] = (jlong)res[s].first_frame;
            }
        if (sg) (*env)->ReleaseLongArrayElements(env, seg_longs, sg, 0);
        if (si) (*env)->ReleaseIntArrayElements(env, seg_ints, si, 0);
    }
    free(res);
    if (check(env, rc) < 0) return 0;
    return (jlong)total;
}

/* ---- the write side (HipFrameStamper) ------------------------------------------------------------ */
JNIEXPORT void JNICALL CLS(stampHost0)(JNIEnv* env, jclass c, jlong ctx, jobject buf, jlong buf_len, jlongArray off,
                                       jintArray len, jint n) {
    (void)c;
    uint8_t* base = buf ? (uint8_t*)(*env)->GetDirectBufferAddress(env, buf) : NULL;
    const jlong capb = buf ? (*env)->GetDirectBufferCapacity(env, buf) : -1;
    if (!base || buf_len < 0 || capb < buf_len || n < 0) {
        throw_arg(env, "stampFrames: not a direct buffer, bufLen beyond it, or n < 0");
        return;
    }
    if (n == 0) return;
    if (!has_len(env, off, n, "off shorter than n") || !has_len(env, len, n, "len shorter than n")) return;
    jlong* o = (*env)->GetLongArrayElements(env, off, NULL);
    jint* l = o ? (*env)->GetIntArrayElements(env, len, NULL) : NULL;
    int rc = RH_E_NOMEM;
    if (o && l)
        rc = rh_crc32c_stamp_host(C(ctx), base, (uint64_t)buf_len, (const uint64_t*)o, (const uint32_t*)l, (uint64_t)n);
    if (l) (*env)->ReleaseIntArrayElements(env, len, l, JNI_ABORT);
    if (o) (*env)->ReleaseLongArrayElements(env, off, o, JNI_ABORT);
    check(env, rc);
}

JNIEXPORT void JNICALL CLS(hostRegister0)(JNIEnv* env, jclass c, jlong ctx, jobject buf) {
    (void)c;
    void* base = buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL;
    const jlong capb = buf ? (*env)->GetDirectBufferCapacity(env, buf) : -1;
    if (!base || capb <= 0) {
        throw_arg(env, "register: not a direct buffer");
        return;
    }
    check(env, rh_host_register(C(ctx), base, (uint64_t)capb));
}

JNIEXPORT void JNICALL CLS(hostUnregister0)(JNIEnv* env, jclass c, jlong ctx, jobject buf) {
    (void)c;
    void* base = buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL;
    if (!base) {
        throw_arg(env, "unregister: not a direct buffer");
        return;
    }
    check(env, rh_host_unregister(C(ctx), base));
}
