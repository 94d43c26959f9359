/*
 * TEST INFRASTRUCTURE ONLY: a JNIEnv without a JVM, so that java/ratis-hip/src/main/native/
 * ratis_hip_jni.c -- compiled into this library unchanged, against tests/jni_stub/jni.h -- runs
 * for real under ctypes (tests/test_gpu_jni.py).  Java arrays and direct buffers are views of
 * caller-owned memory (numpy arrays): Get*ArrayElements / GetPrimitiveArrayCritical hand out the
 * memory itself (no copies, so a Release with JNI_ABORT cannot hide a write the glue made), region
 * calls copy, NewDirectByteBuffer wraps a pointer, and ThrowNew records the exception the glue
 * raises (class name + message) for the test to read back -- the mapping RatisHip.java documents.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"

enum { FJ_ARRAY = 1, FJ_BUFFER = 2, FJ_CLASS = 3 };

struct _jobject {
    int kind;
    int elem;      /* FJ_ARRAY: element size in bytes                        */
    jsize len;     /* FJ_ARRAY: elements                                     */
    void* data;    /* FJ_ARRAY: elements; FJ_BUFFER: address                 */
    jlong cap;     /* FJ_BUFFER: capacity in bytes                           */
    char name[96]; /* FJ_CLASS                                               */
};

static char g_exc_class[96];
static char g_exc_msg[512];
static int g_exc_pending;
static long g_calls_get, g_calls_release;   /* element / critical pins handed out and given back */

static jclass fj_FindClass(JNIEnv* env, const char* name) {
    (void)env;
    struct _jobject* o = (struct _jobject*)calloc(1, sizeof(*o));
    o->kind = FJ_CLASS;
    snprintf(o->name, sizeof(o->name), "%s", name);
    return o;   /* leaked on purpose: a handful per test */
}

static jint fj_ThrowNew(JNIEnv* env, jclass c, const char* msg) {
    (void)env;
    if (!g_exc_pending) {   /* the first exception wins, as in a JVM */
        snprintf(g_exc_class, sizeof(g_exc_class), "%s", c ? c->name : "?");
        snprintf(g_exc_msg, sizeof(g_exc_msg), "%s", msg ? msg : "");
        g_exc_pending = 1;
    }
    return 0;
}

static jsize fj_GetArrayLength(JNIEnv* env, jarray a) {
    (void)env;
    return a->len;
}

static void region(jarray a, jsize start, jsize n, void* dst, const void* src) {
    if (start < 0 || n < 0 || start + n > a->len) {
        if (!g_exc_pending) {
            strcpy(g_exc_class, "java/lang/ArrayIndexOutOfBoundsException");
            strcpy(g_exc_msg, "region outside the array");
            g_exc_pending = 1;
        }
        return;
    }
    if (dst) memcpy(dst, (char*)a->data + (size_t)start * a->elem, (size_t)n * a->elem);
    else memcpy((char*)a->data + (size_t)start * a->elem, src, (size_t)n * a->elem);
}

static void fj_GetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize s, jsize n, jbyte* buf) {
    (void)env;
    region(a, s, n, buf, NULL);
}
static void fj_SetIntArrayRegion(JNIEnv* env, jintArray a, jsize s, jsize n, const jint* buf) {
    (void)env;
    region(a, s, n, NULL, buf);
}
static void fj_SetLongArrayRegion(JNIEnv* env, jlongArray a, jsize s, jsize n, const jlong* buf) {
    (void)env;
    region(a, s, n, NULL, buf);
}
static void fj_SetBooleanArrayRegion(JNIEnv* env, jbooleanArray a, jsize s, jsize n, const jboolean* buf) {
    (void)env;
    region(a, s, n, NULL, buf);
}
static void* pin(jarray a, jboolean* is_copy) {
    if (is_copy) *is_copy = JNI_FALSE;
    ++g_calls_get;
    return a->data;
}
static jint* fj_GetIntArrayElements(JNIEnv* env, jintArray a, jboolean* c) {
    (void)env;
    return (jint*)pin(a, c);
}
static jlong* fj_GetLongArrayElements(JNIEnv* env, jlongArray a, jboolean* c) {
    (void)env;
    return (jlong*)pin(a, c);
}
static void fj_ReleaseIntArrayElements(JNIEnv* env, jintArray a, jint* p, jint mode) {
    (void)env, (void)a, (void)p, (void)mode;
    ++g_calls_release;
}
static void fj_ReleaseLongArrayElements(JNIEnv* env, jlongArray a, jlong* p, jint mode) {
    (void)env, (void)a, (void)p, (void)mode;
    ++g_calls_release;
}
static void* fj_GetPrimitiveArrayCritical(JNIEnv* env, jarray a, jboolean* c) {
    (void)env;
    return pin(a, c);
}
static void fj_ReleasePrimitiveArrayCritical(JNIEnv* env, jarray a, void* p, jint mode) {
    (void)env, (void)a, (void)p, (void)mode;
    ++g_calls_release;
}
static jobject fj_NewDirectByteBuffer(JNIEnv* env, void* addr, jlong cap) {
    (void)env;
    struct _jobject* o = (struct _jobject*)calloc(1, sizeof(*o));
    o->kind = FJ_BUFFER;
    o->data = addr;
    o->cap = cap;
    return o;
}
static void* fj_GetDirectBufferAddress(JNIEnv* env, jobject b) {
    (void)env;
    return (b && b->kind == FJ_BUFFER) ? b->data : NULL;   /* NULL for a heap buffer, as the JVM */
}
static jlong fj_GetDirectBufferCapacity(JNIEnv* env, jobject b) {
    (void)env;
    return (b && b->kind == FJ_BUFFER) ? b->cap : -1;
}
static jboolean fj_ExceptionCheck(JNIEnv* env) {
    (void)env;
    return g_exc_pending ? JNI_TRUE : JNI_FALSE;
}

static const struct JNINativeInterface_ g_table = {
    fj_FindClass, fj_ThrowNew, fj_GetArrayLength, fj_GetByteArrayRegion, fj_SetIntArrayRegion,
    fj_SetLongArrayRegion, fj_SetBooleanArrayRegion, fj_GetIntArrayElements, fj_GetLongArrayElements,
    fj_ReleaseIntArrayElements, fj_ReleaseLongArrayElements, fj_GetPrimitiveArrayCritical,
    fj_ReleasePrimitiveArrayCritical, fj_NewDirectByteBuffer, fj_GetDirectBufferAddress,
    fj_GetDirectBufferCapacity, fj_ExceptionCheck,
};
static JNIEnv g_env = &g_table;

/* ---- ctypes side ------------------------------------------------------------------------------ */
JNIEXPORT JNIEnv* fj_env(void) { return &g_env; }

/* A Java array of `len` elements of `elem` bytes over caller memory (NULL data: a null reference). */
JNIEXPORT jobject fj_array(int elem, jsize len, void* data) {
    struct _jobject* o = (struct _jobject*)calloc(1, sizeof(*o));
    o->kind = FJ_ARRAY;
    o->elem = elem;
    o->len = len;
    o->data = data;
    return o;
}

/* A direct ByteBuffer over caller memory; kind = 0 makes a heap buffer (no address). */
JNIEXPORT jobject fj_buffer(void* addr, jlong cap, int direct) {
    struct _jobject* o = (struct _jobject*)calloc(1, sizeof(*o));
    o->kind = direct ? FJ_BUFFER : FJ_ARRAY;
    o->data = addr;
    o->cap = cap;
    return o;
}

JNIEXPORT void* fj_buffer_address(jobject b) { return b ? b->data : NULL; }
JNIEXPORT jlong fj_buffer_capacity(jobject b) { return b ? b->cap : -1; }

JNIEXPORT void fj_free(jobject o) { free(o); }

/* 1 and the exception (class, message) when one is pending; clears it. */
JNIEXPORT int fj_take_exception(char* cls, int cls_len, char* msg, int msg_len) {
    if (!g_exc_pending) return 0;
    snprintf(cls, (size_t)cls_len, "%s", g_exc_class);
    snprintf(msg, (size_t)msg_len, "%s", g_exc_msg);
    g_exc_pending = 0;
    g_exc_class[0] = g_exc_msg[0] = 0;
    return 1;
}

/* Pins handed out minus pins given back (the glue must release every array it pinned). */
JNIEXPORT long fj_pins_outstanding(void) { return g_calls_get - g_calls_release; }
