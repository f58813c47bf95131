/*
 * jni_harness.c — drives jvm/native/fsm_jni.c without a JVM (TEST
 * INFRASTRUCTURE).  Objects are tagged heap blocks; FindClass / ThrowNew record
 * the pending exception the way the JVM would.  harness_spade / harness_tsr
 * call the JNI entry points like FsmNativeJNI.spade / .tsr and render the result
 * exactly as GpuSPADE / GpuTSR (jvm/scala) map it: one GpuPattern.serialize()
 * line per pattern, one "X ==> Y #SUP: s #CONF: c" line per rule, or
 * "EXCEPTION java/lang/Exception: <message>" when the shim threw.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"

enum { K_CLASS, K_STR, K_INT, K_LONG, K_DOUBLE, K_OBJ };
struct _jobject {
    int kind;
    jsize len;
    void* data;
};

static char g_exc[2048];
static int g_has_exc;

static jobject mk(int kind, jsize len, size_t elem) {
    struct _jobject* o = calloc(1, sizeof *o);
    o->kind = kind;
    o->len = len;
    o->data = calloc((size_t)(len > 0 ? len : 1), elem);
    return o;
}
static jclass FindClass(JNIEnv* e, const char* n) {
    (void)e;
    jobject o = mk(K_CLASS, (jsize)strlen(n) + 1, 1);
    memcpy(o->data, n, strlen(n) + 1);
    return o;
}
static jint ThrowNew(JNIEnv* e, jclass c, const char* m) {
    (void)e;
    snprintf(g_exc, sizeof g_exc, "%s: %s", (const char*)c->data, m);
    g_has_exc = 1;
    return 0;
}
static void DeleteLocalRef(JNIEnv* e, jobject o) { (void)e; (void)o; }
static jsize GetArrayLength(JNIEnv* e, jarray a) { (void)e; return a->len; }
static jint* GetIntArrayElements(JNIEnv* e, jintArray a, jboolean* c) {
    (void)e;
    if (c) *c = 0;
    return (jint*)a->data;
}
static void ReleaseIntArrayElements(JNIEnv* e, jintArray a, jint* p, jint m) { (void)e; (void)a; (void)p; (void)m; }
static jobject GetObjectArrayElement(JNIEnv* e, jobjectArray a, jsize i) { (void)e; return ((jobject*)a->data)[i]; }
static void SetObjectArrayElement(JNIEnv* e, jobjectArray a, jsize i, jobject v) { (void)e; ((jobject*)a->data)[i] = v; }
static const char* GetStringUTFChars(JNIEnv* e, jstring s, jboolean* c) {
    (void)e;
    if (c) *c = 0;
    return (const char*)s->data;
}
static void ReleaseStringUTFChars(JNIEnv* e, jstring s, const char* p) { (void)e; (void)s; (void)p; }
static jintArray NewIntArray(JNIEnv* e, jsize n) { (void)e; return mk(K_INT, n, sizeof(jint)); }
static jlongArray NewLongArray(JNIEnv* e, jsize n) { (void)e; return mk(K_LONG, n, sizeof(jlong)); }
static jdoubleArray NewDoubleArray(JNIEnv* e, jsize n) { (void)e; return mk(K_DOUBLE, n, sizeof(jdouble)); }
static jobjectArray NewObjectArray(JNIEnv* e, jsize n, jclass c, jobject init) {
    (void)e; (void)c; (void)init;
    return mk(K_OBJ, n, sizeof(jobject));
}
static void SetIntArrayRegion(JNIEnv* e, jintArray a, jsize s, jsize n, const jint* b) {
    (void)e;
    memcpy((jint*)a->data + s, b, sizeof(jint) * (size_t)n);
}
static void SetLongArrayRegion(JNIEnv* e, jlongArray a, jsize s, jsize n, const jlong* b) {
    (void)e;
    memcpy((jlong*)a->data + s, b, sizeof(jlong) * (size_t)n);
}
static void SetDoubleArrayRegion(JNIEnv* e, jdoubleArray a, jsize s, jsize n, const jdouble* b) {
    (void)e;
    memcpy((jdouble*)a->data + s, b, sizeof(jdouble) * (size_t)n);
}

static const struct JNINativeInterface_ g_table = {
    FindClass, ThrowNew, DeleteLocalRef, GetArrayLength, GetIntArrayElements, ReleaseIntArrayElements,
    GetObjectArrayElement, SetObjectArrayElement, GetStringUTFChars, ReleaseStringUTFChars, NewIntArray,
    NewLongArray, NewDoubleArray, NewObjectArray, SetIntArrayRegion, SetLongArrayRegion, SetDoubleArrayRegion};
static JNIEnv g_env = &g_table;

jobjectArray Java_de_kp_spark_fsm_gpu_FsmNativeJNI_spade(JNIEnv*, jclass, jintArray, jobjectArray, jdouble, jboolean,
                                                        jintArray);
jobjectArray Java_de_kp_spark_fsm_gpu_FsmNativeJNI_tsr(JNIEnv*, jclass, jintArray, jobjectArray, jint, jdouble, jintArray);

/* FsmNative.devices as the Scala side passes it: ndev ordinals */
static jintArray device_list(int ndev, const int* devs) {
    jintArray a = NewIntArray(&g_env, ndev);
    SetIntArrayRegion(&g_env, a, 0, ndev, devs);
    return a;
}

static void inputs(int n, const int* sids, const char** lines, jintArray* js, jobjectArray* jl) {
    *js = NewIntArray(&g_env, n);
    SetIntArrayRegion(&g_env, *js, 0, n, sids);
    *jl = NewObjectArray(&g_env, n, NULL, NULL);
    for (int i = 0; i < n; ++i) {
        jobject s = mk(K_STR, (jsize)strlen(lines[i]) + 1, 1);
        memcpy(s->data, lines[i], strlen(lines[i]) + 1);
        SetObjectArrayElement(&g_env, *jl, i, s);
    }
}

typedef struct {
    char* p;
    size_t n, cap;
} buf_t;
static void put(buf_t* b, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
#include <stdarg.h>
static void put(buf_t* b, const char* fmt, ...) {
    va_list ap;
    for (;;) {
        va_start(ap, fmt);
        const int k = vsnprintf(b->p + b->n, b->cap - b->n, fmt, ap);
        va_end(ap);
        if (k >= 0 && b->n + (size_t)k < b->cap) {
            b->n += (size_t)k;
            return;
        }
        b->cap = b->cap * 2 + (size_t)k + 64;
        b->p = realloc(b->p, b->cap);
    }
}

/* GpuSPADE.extractRDDPatterns' mapping, rendered as GpuPattern.serialize() lines */
char* harness_spade(int n, const int* sids, const char** lines, double support, int ndev, const int* devs) {
    jintArray js;
    jobjectArray jl;
    inputs(n, sids, lines, &js, &jl);
    g_has_exc = 0;
    jobjectArray res =
        Java_de_kp_spark_fsm_gpu_FsmNativeJNI_spade(&g_env, NULL, js, jl, support, 1, device_list(ndev, devs));
    buf_t b = {malloc(256), 0, 256};
    b.p[0] = 0;
    if (g_has_exc || !res) {
        put(&b, "EXCEPTION %s", g_has_exc ? g_exc : "(null result without exception)");
        return b.p;
    }
    jobject* parts = (jobject*)res->data;
    const jint* sup = parts[0]->data;
    const jlong *po = parts[1]->data, *so = parts[2]->data;
    const jint* it = parts[3]->data;
    for (jsize p = 0; p < parts[0]->len; ++p) {
        for (jlong s = po[p]; s < po[p + 1]; ++s) {
            for (jlong q = so[s]; q < so[s + 1]; ++q) put(&b, q > so[s] ? " %d" : "%d", it[q]);
            put(&b, " -1 ");
        }
        put(&b, "| %d\n", sup[p]);
    }
    return b.p;
}

/* GpuTSR.extractRDDRules' mapping, one GpuRule.toString line per rule (%.17g confidence) */
char* harness_tsr(int n, const int* sids, const char** lines, int k, double minconf, int ndev, const int* devs) {
    jintArray js;
    jobjectArray jl;
    inputs(n, sids, lines, &js, &jl);
    g_has_exc = 0;
    jobjectArray res = Java_de_kp_spark_fsm_gpu_FsmNativeJNI_tsr(&g_env, NULL, js, jl, k, minconf, device_list(ndev, devs));
    buf_t b = {malloc(256), 0, 256};
    b.p[0] = 0;
    if (g_has_exc || !res) {
        put(&b, "EXCEPTION %s", g_has_exc ? g_exc : "(null result without exception)");
        return b.p;
    }
    jobject* parts = (jobject*)res->data;
    const jint* sup = parts[0]->data;
    const jdouble* conf = parts[1]->data;
    const jlong *ao = parts[2]->data, *co = parts[4]->data;
    const jint *a = parts[3]->data, *c = parts[5]->data;
    for (jsize q = 0; q < parts[0]->len; ++q) {
        for (jlong i = ao[q]; i < ao[q + 1]; ++i) put(&b, i > ao[q] ? ",%d" : "%d", a[i]);
        put(&b, " ==> ");
        for (jlong i = co[q]; i < co[q + 1]; ++i) put(&b, i > co[q] ? ",%d" : "%d", c[i]);
        put(&b, " #SUP: %d #CONF: %.17g\n", sup[q], conf[q]);
    }
    return b.p;
}

void harness_free(char* p) { free(p); }
