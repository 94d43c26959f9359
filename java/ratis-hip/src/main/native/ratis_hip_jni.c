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
 * IOException, message = rh_last_error() (thread-local in the library).
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ratis_hip.h"

#define CLS(name) Java_org_apache_ratis_hip_RatisHip_##name

static void throw_rh(JNIEnv* env, int rc) {
    const char* cls = (rc == RH_E_INVAL || rc == RH_E_RANGE) ? "java/lang/IllegalArgumentException"
                                                             : "java/io/IOException";
    jclass c = (*env)->FindClass(env, cls);
    if (c) (*env)->ThrowNew(env, c, rh_last_error());
}

static int check(JNIEnv* env, int rc) {
    if (rc < 0) throw_rh(env, rc);
    return rc;
}

static rh_node* N(jlong h) { return (rh_node*)(intptr_t)h; }

static rh_groups* shard_table(JNIEnv* env, jlong node, jint shard) {
    rh_groups* g = rh_node_groups(N(node), (int)shard);
    if (!g) {
        jclass c = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
        if (c) (*env)->ThrowNew(env, c, "no such shard");
    }
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
        const jsize n = (*env)->GetArrayLength(env, src);
        for (int k = 0; k < (int)RH_MAX_FOLLOWERS; ++k) map[k] = -1;
        (*env)->GetByteArrayRegion(env, src, 0, n < (jsize)RH_MAX_FOLLOWERS ? n : (jsize)RH_MAX_FOLLOWERS,
                                   (jbyte*)map);
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
    const rh_delta* d = (const rh_delta*)(*env)->GetDirectBufferAddress(env, direct);
    if (!d && n) {
        throw_rh(env, RH_E_INVAL);
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
    rh_groups* g = shard_table(env, node, shard);
    if (g) check(env, rh_deltas_submit(g, (size_t)n));
}

JNIEXPORT jlong JNICALL CLS(commitBatch0)(JNIEnv* env, jclass c, jlong node, jintArray adv_slot,
                                          jlongArray adv_commit, jintArray wall_slot, jlongArray wall_min) {
    (void)c;
    const jsize acap = adv_slot ? (*env)->GetArrayLength(env, adv_slot) : 0;
    const jsize wcap = wall_slot ? (*env)->GetArrayLength(env, wall_slot) : 0;
    rh_index_event* adv = (rh_index_event*)malloc(sizeof(rh_index_event) * (size_t)(acap ? acap : 1));
    rh_index_event* wall = (rh_index_event*)malloc(sizeof(rh_index_event) * (size_t)(wcap ? wcap : 1));
    uint64_t na = 0, nw = 0;
    const uint32_t flags = wall_slot ? RH_COMMIT_WATCH_ALL : 0u;   /* watch-ALL levels only when asked */
    int rc = (adv && wall) ? rh_node_commit_batch(N(node), flags, adv, (uint64_t)acap, &na, wall, (uint64_t)wcap, &nw)
                           : RH_E_NOMEM;
    if (rc >= 0) {
        const jsize ka = (jsize)(na < (uint64_t)acap ? na : (uint64_t)acap);
        const jsize kw = (jsize)(nw < (uint64_t)wcap ? nw : (uint64_t)wcap);
        jint* s = ka ? (*env)->GetPrimitiveArrayCritical(env, adv_slot, NULL) : NULL;
        jlong* v = ka ? (*env)->GetPrimitiveArrayCritical(env, adv_commit, NULL) : NULL;
        for (jsize i = 0; i < ka; ++i) {
            s[i] = (jint)adv[i].slot;
            v[i] = (jlong)adv[i].value;
        }
        if (v) (*env)->ReleasePrimitiveArrayCritical(env, adv_commit, v, 0);
        if (s) (*env)->ReleasePrimitiveArrayCritical(env, adv_slot, s, 0);
        s = kw ? (*env)->GetPrimitiveArrayCritical(env, wall_slot, NULL) : NULL;
        v = kw ? (*env)->GetPrimitiveArrayCritical(env, wall_min, NULL) : NULL;
        for (jsize i = 0; i < kw; ++i) {
            s[i] = (jint)wall[i].slot;
            v[i] = (jlong)wall[i].value;
        }
        if (v) (*env)->ReleasePrimitiveArrayCritical(env, wall_min, v, 0);
        if (s) (*env)->ReleasePrimitiveArrayCritical(env, wall_slot, s, 0);
    }
    free(adv);
    free(wall);
    if (check(env, rc) < 0) return 0;
    return (jlong)((na << 32) | (nw & 0xFFFFFFFFull));
}

JNIEXPORT jint JNICALL CLS(watchLevels0)(JNIEnv* env, jclass c, jlong node, jint shard, jintArray slot,
                                         jlongArray mn, jlongArray mj, jlongArray mx, jbooleanArray valid) {
    (void)c;
    rh_groups* g = shard_table(env, node, shard);
    if (!g) return 0;
    const rh_watch_event* ev = NULL;
    uint64_t n = 0;
    if (check(env, rh_watch_levels(g, &ev, &n)) < 0) return 0;
    const jsize cap = (*env)->GetArrayLength(env, slot);
    const jsize k = (jsize)(n < (uint64_t)cap ? n : (uint64_t)cap);
    for (jsize i = 0; i < k; ++i) {
        const jint s = (jint)ev[i].slot;
        const jlong a = (jlong)ev[i].min, b = (jlong)ev[i].majority, d = (jlong)ev[i].max;
        const jboolean v = ev[i].valid ? JNI_TRUE : JNI_FALSE;
        (*env)->SetIntArrayRegion(env, slot, i, 1, &s);
        (*env)->SetLongArrayRegion(env, mn, i, 1, &a);
        (*env)->SetLongArrayRegion(env, mj, i, 1, &b);
        (*env)->SetLongArrayRegion(env, mx, i, 1, &d);
        (*env)->SetBooleanArrayRegion(env, valid, i, 1, &v);
    }
    return (jint)n;
}

JNIEXPORT void JNICALL CLS(leaseStart0)(JNIEnv* env, jclass c, jlong node, jint slot, jlong now, jboolean enabled) {
    (void)c;
    check(env, rh_node_group_lease_start(N(node), (uint32_t)slot, (int64_t)now, enabled ? 1 : 0));
}

JNIEXPORT void JNICALL CLS(leaseBatch0)(JNIEnv* env, jclass c, jlong node, jlong now, jlong timeout_ms,
                                        jlongArray bits) {
    (void)c;
    const jsize n = (*env)->GetArrayLength(env, bits);
    jlong* b = (*env)->GetLongArrayElements(env, bits, NULL);
    if (!b) return;
    const int rc = rh_node_lease_batch(N(node), (int64_t)now, (int64_t)timeout_ms, (uint64_t*)b, (uint64_t)n);
    (*env)->ReleaseLongArrayElements(env, bits, b, rc < 0 ? JNI_ABORT : 0);
    check(env, rc);
}

JNIEXPORT jlong JNICALL CLS(verifyHost0)(JNIEnv* env, jclass c, jlong node, jint shard, jobject seg, jlong len,
                                         jlongArray off, jintArray flen, jint n, jintArray crc, jlongArray bad) {
    (void)c;
    rh_ctx* ctx = rh_node_ctx(N(node), (int)shard);
    const uint8_t* p = (const uint8_t*)(*env)->GetDirectBufferAddress(env, seg);
    if (!ctx || (!p && len)) {
        throw_rh(env, RH_E_INVAL);
        return 0;
    }
    jlong* o = (*env)->GetLongArrayElements(env, off, NULL);
    jint* l = (*env)->GetIntArrayElements(env, flen, NULL);
    jint* cr = crc ? (*env)->GetIntArrayElements(env, crc, NULL) : NULL;
    jlong* b = bad ? (*env)->GetLongArrayElements(env, bad, NULL) : NULL;
    uint64_t nb = 0;
    const int rc = rh_crc32c_verify_host(ctx, p, (uint64_t)len, (const uint64_t*)o, (const uint32_t*)l, (uint64_t)n,
                                         (uint32_t*)cr, (uint64_t*)b, &nb);
    if (b) (*env)->ReleaseLongArrayElements(env, bad, b, 0);
    if (cr) (*env)->ReleaseIntArrayElements(env, crc, cr, 0);
    (*env)->ReleaseIntArrayElements(env, flen, l, JNI_ABORT);
    (*env)->ReleaseLongArrayElements(env, off, o, JNI_ABORT);
    if (check(env, rc) < 0) return 0;
    return (jlong)nb;
}
