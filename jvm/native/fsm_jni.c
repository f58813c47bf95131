/*
 * fsm_jni.c — JNI glue between the Scala drop-in bodies (jvm/scala/...) and
 * libfsm.so (include/fsm.h).  Replaces, for the JVM side, the bodies of
 *   SPADE.extractRDDPatterns   /root/reference/src/main/scala/de/kp/spark/fsm/SPADE.scala:36
 *   TSR.extractRDDRules        /root/reference/src/main/scala/de/kp/spark/fsm/TSR.scala:31
 * (see GpuSPADE.scala / GpuTSR.scala).  Every failure is thrown as a
 * java.lang.Exception, never an Error: TrainActor only catches Exception
 * (actor/TrainActor.scala:66), so anything else would leave the request stuck
 * at MINING_STARTED.
 *
 * Build on a JVM box (this image has no JDK):
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux \
 *       -I../../include fsm_jni.c -L../../spark-fsm_amd/spark_fsm_amd -lfsm -o libfsm_jni.so
 * tests/test_jvm_shim.py compiles it here against a minimal jni.h and drives
 * it through an in-process JNIEnv (tests/jni_harness.c).
 */
#include <jni.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fsm.h"

static void throw_exception(JNIEnv* env, const char* what, int rc, const char* detail) {
    char msg[1024];
    snprintf(msg, sizeof msg, "libfsm %s failed (FSM error %d): %s", what, rc, detail ? detail : "");
    jclass ex = (*env)->FindClass(env, "java/lang/Exception");
    if (ex) (*env)->ThrowNew(env, ex, msg);
}

/* Collects the RDD's (sid, line) records the Scala side passes as arrays and
 * builds the flattened DB (parse + flatten + upload once).  NULL after a throw. */
static fsm_db* make_db(JNIEnv* env, fsm_ctx* ctx, int32_t mode, jintArray jsids, jobjectArray jlines, int* rc_out) {
    const jsize n = (*env)->GetArrayLength(env, jsids);
    if ((*env)->GetArrayLength(env, jlines) != n) {
        *rc_out = FSM_EINVAL;
        throw_exception(env, "fsm_db_from_spmf", FSM_EINVAL, "sids and lines differ in length");
        return NULL;
    }
    jint* sids = (*env)->GetIntArrayElements(env, jsids, NULL);
    const char** lines = malloc(sizeof(char*) * (size_t)(n ? n : 1));
    int64_t* lens = malloc(sizeof(int64_t) * (size_t)(n ? n : 1));
    jstring* refs = malloc(sizeof(jstring) * (size_t)(n ? n : 1));
    if (!sids || !lines || !lens || !refs) {
        if (sids) (*env)->ReleaseIntArrayElements(env, jsids, sids, JNI_ABORT);
        free(lines);
        free(lens);
        free(refs);
        *rc_out = FSM_ENOMEM;
        throw_exception(env, "fsm_db_from_spmf", FSM_ENOMEM, "host allocation failed");
        return NULL;
    }
    jsize got = 0;
    for (; got < n; ++got) {
        refs[got] = (jstring)(*env)->GetObjectArrayElement(env, jlines, got);
        lines[got] = refs[got] ? (*env)->GetStringUTFChars(env, refs[got], NULL) : NULL;
        if (!lines[got]) break;
        lens[got] = (int64_t)strlen(lines[got]);
    }
    fsm_db* db = NULL;
    int rc = FSM_EINVAL;
    if (got == n) rc = fsm_db_from_spmf(ctx, mode, (const int32_t*)sids, lines, lens, n, &db);
    for (jsize i = 0; i < got; ++i) {
        (*env)->ReleaseStringUTFChars(env, refs[i], lines[i]);
        (*env)->DeleteLocalRef(env, refs[i]);
    }
    (*env)->ReleaseIntArrayElements(env, jsids, sids, JNI_ABORT);
    free(lines);
    free(lens);
    free(refs);
    *rc_out = got != n ? FSM_EINVAL : rc;
    if (got != n) {
        throw_exception(env, "fsm_db_from_spmf", FSM_EINVAL, "a null line in the dataset");
        return NULL;
    }
    if (rc != FSM_OK) {
        throw_exception(env, "fsm_db_from_spmf", rc, fsm_last_error(ctx));
        return NULL;
    }
    return db;
}

/* The request's device list (FsmNative.devices, -Dfsm.devices).  One entry: the single-GPU
 * context on that device.  More: ONE context that shards the mine over in-process ranks,
 * rank r on devices[r] (fsm_opts.ndevices): the Spark driver thread
 * (SPADE.scala:132-133, TSR.scala:102-103) makes one call and gets the whole result back. */
typedef struct {
    int32_t nd;
    int32_t dev[FSM_MAX_DEVICES];
} dev_list;

/* Idle contexts kept between requests, keyed by device list: a context (and, for a device
 * list, its rank threads, HIP streams, pools and pinned staging) is made once, not per
 * request (each actor is per request and stops afterwards, FSMMiner.scala:77-83, but the
 * process stays).  Concurrent requests take distinct contexts.  A context whose call failed
 * with FSM_ECOMM / FSM_EDEVICE / FSM_ENOMEM is destroyed, not kept. */
#define CTX_POOL_MAX 4
static struct {
    fsm_ctx* ctx;
    dev_list dl;
} g_idle[CTX_POOL_MAX];
static int g_nidle;
static pthread_mutex_t g_idle_mu = PTHREAD_MUTEX_INITIALIZER;

static int same_devices(const dev_list* a, const dev_list* b) {
    return a->nd == b->nd && memcmp(a->dev, b->dev, sizeof(int32_t) * (size_t)a->nd) == 0;
}

static fsm_ctx* make_ctx(JNIEnv* env, jintArray jdevices, dev_list* dl) {
    memset(dl, 0, sizeof *dl);
    const jsize nd = jdevices ? (*env)->GetArrayLength(env, jdevices) : 0;
    if (nd > FSM_MAX_DEVICES) {
        throw_exception(env, "fsm_ctx_create", FSM_EINVAL, "more devices than FSM_MAX_DEVICES");
        return NULL;
    }
    if (nd > 0) {
        jint* dv = (*env)->GetIntArrayElements(env, jdevices, NULL);
        if (!dv) {
            throw_exception(env, "fsm_ctx_create", FSM_ENOMEM, "device list unavailable");
            return NULL;
        }
        dl->nd = nd;
        for (jsize r = 0; r < nd; ++r) dl->dev[r] = dv[r];
        (*env)->ReleaseIntArrayElements(env, jdevices, dv, JNI_ABORT);
    }
    pthread_mutex_lock(&g_idle_mu);
    for (int i = 0; i < g_nidle; ++i)
        if (same_devices(&g_idle[i].dl, dl)) {
            fsm_ctx* ctx = g_idle[i].ctx;
            g_idle[i] = g_idle[--g_nidle];
            pthread_mutex_unlock(&g_idle_mu);
            return ctx;
        }
    pthread_mutex_unlock(&g_idle_mu);
    fsm_opts o;
    memset(&o, 0, sizeof o);
    o.nranks = 1;
    if (dl->nd > 0) o.device = dl->dev[0];
    if (dl->nd > 1) {
        o.ndevices = dl->nd;
        for (int32_t r = 0; r < dl->nd; ++r) o.devices[r] = dl->dev[r];
    }
    fsm_ctx* ctx = NULL;
    const int rc = fsm_ctx_create(&o, &ctx);
    if (rc != FSM_OK) {
        throw_exception(env, "fsm_ctx_create", rc, fsm_last_error(NULL));
        return NULL;
    }
    return ctx;
}

/* back to the idle list after a request (rc: the request's last libfsm status) */
static void release_ctx(fsm_ctx* ctx, const dev_list* dl, int rc) {
    if (!ctx) return;
    if (rc == FSM_OK || rc == FSM_EINVAL || rc == FSM_EPARSE || rc == FSM_ELIMIT) {
        pthread_mutex_lock(&g_idle_mu);
        if (g_nidle < CTX_POOL_MAX) {
            g_idle[g_nidle].ctx = ctx;
            g_idle[g_nidle].dl = *dl;
            ++g_nidle;
            ctx = NULL;
        }
        pthread_mutex_unlock(&g_idle_mu);
    }
    if (ctx) fsm_ctx_destroy(ctx);
}

/* FsmNativeJNI.release(): destroy the idle contexts (the Scala side calls it at shutdown) */
JNIEXPORT void JNICALL Java_de_kp_spark_fsm_gpu_FsmNativeJNI_release(JNIEnv* env, jclass cls) {
    (void)env;
    (void)cls;
    pthread_mutex_lock(&g_idle_mu);
    const int n = g_nidle;
    fsm_ctx* keep[CTX_POOL_MAX];
    for (int i = 0; i < n; ++i) keep[i] = g_idle[i].ctx;
    g_nidle = 0;
    pthread_mutex_unlock(&g_idle_mu);
    for (int i = 0; i < n; ++i) fsm_ctx_destroy(keep[i]);
}

/* de.kp.spark.fsm.gpu.FsmNativeJNI.spade(int[] sids, String[] lines, double support, boolean dfs,
 *                                        int[] devices): Object[] =
 *   [support: Array[Int], patOff: Array[Long], setOff: Array[Long], items: Array[Int], total+minsup: Array[Long]] */
JNIEXPORT jobjectArray JNICALL Java_de_kp_spark_fsm_gpu_FsmNativeJNI_spade(JNIEnv* env, jclass cls, jintArray jsids,
                                                                       jobjectArray jlines, jdouble support,
                                                                       jboolean dfs, jintArray jdevices) {
    (void)cls;
    dev_list dl;
    fsm_ctx* ctx = make_ctx(env, jdevices, &dl);
    if (!ctx) return NULL;
    jobjectArray res = NULL;
    int rc = FSM_OK;
    fsm_db* db = make_db(env, ctx, FSM_MODE_SPADE, jsids, jlines, &rc);
    fsm_patterns* p = NULL;
    if (db) {
        /* dfs as SpadeAlgorithm(support, dfs) takes it (SPADE.scala:132); SPADEActor passes the
         * default true (SPADE.scala:36, SPADEActor.scala:47) */
        rc = fsm_spade_mine(ctx, db, support, dfs ? 1 : 0, &p);
        if (rc != FSM_OK) throw_exception(env, "fsm_spade_mine", rc, fsm_last_error(ctx));
    }
    if (p) {
        jintArray sup = (*env)->NewIntArray(env, (jsize)p->n);
        jlongArray po = (*env)->NewLongArray(env, (jsize)(p->n + 1));
        jlongArray so = (*env)->NewLongArray(env, (jsize)(p->n_sets + 1));
        jintArray it = (*env)->NewIntArray(env, (jsize)p->n_items);
        jlongArray meta = (*env)->NewLongArray(env, 2);
        jclass obj = (*env)->FindClass(env, "java/lang/Object");
        if (sup && po && so && it && meta && obj) {
            const jlong m[2] = {(jlong)p->total, (jlong)p->minsup};
            (*env)->SetIntArrayRegion(env, sup, 0, (jsize)p->n, (const jint*)p->support);
            (*env)->SetLongArrayRegion(env, po, 0, (jsize)(p->n + 1), (const jlong*)p->pat_off);
            (*env)->SetLongArrayRegion(env, so, 0, (jsize)(p->n_sets + 1), (const jlong*)p->set_off);
            (*env)->SetIntArrayRegion(env, it, 0, (jsize)p->n_items, (const jint*)p->items);
            (*env)->SetLongArrayRegion(env, meta, 0, 2, m);
            res = (*env)->NewObjectArray(env, 5, obj, NULL);
            if (res) {
                jobject parts[5] = {sup, po, so, it, meta};
                for (int i = 0; i < 5; ++i) (*env)->SetObjectArrayElement(env, res, i, parts[i]);
            }
        } else {
            throw_exception(env, "result copy", FSM_ENOMEM, "JVM array allocation failed");
        }
        fsm_patterns_free(p);
    }
    fsm_db_free(db);
    release_ctx(ctx, &dl, rc);
    return res;
}

/* FsmNativeJNI.tsr(int[] sids, String[] lines, int k, double minconf, int[] devices): Object[] =
 *   [support: Array[Int], confidence: Array[Double], anteOff: Array[Long], ante: Array[Int],
 *    consOff: Array[Long], cons: Array[Int], total+finalMinsup: Array[Long]] */
JNIEXPORT jobjectArray JNICALL Java_de_kp_spark_fsm_gpu_FsmNativeJNI_tsr(JNIEnv* env, jclass cls, jintArray jsids,
                                                                     jobjectArray jlines, jint k, jdouble minconf,
                                                                     jintArray jdevices) {
    (void)cls;
    dev_list dl;
    fsm_ctx* ctx = make_ctx(env, jdevices, &dl);
    if (!ctx) return NULL;
    jobjectArray res = NULL;
    int rc = FSM_OK;
    fsm_db* db = make_db(env, ctx, FSM_MODE_TSR, jsids, jlines, &rc);
    fsm_rules* r = NULL;
    if (db) {
        rc = fsm_tsr_mine(ctx, db, k, minconf, &r);
        if (rc != FSM_OK) throw_exception(env, "fsm_tsr_mine", rc, fsm_last_error(ctx));
    }
    if (r) {
        const jsize n = (jsize)r->n, na = (jsize)r->ante_off[r->n], nc = (jsize)r->cons_off[r->n];
        jintArray sup = (*env)->NewIntArray(env, n);
        jdoubleArray conf = (*env)->NewDoubleArray(env, n);
        jlongArray ao = (*env)->NewLongArray(env, n + 1), co = (*env)->NewLongArray(env, n + 1);
        jintArray a = (*env)->NewIntArray(env, na), c = (*env)->NewIntArray(env, nc);
        jlongArray meta = (*env)->NewLongArray(env, 2);
        jclass obj = (*env)->FindClass(env, "java/lang/Object");
        if (sup && conf && ao && co && a && c && meta && obj) {
            const jlong m[2] = {(jlong)r->total, (jlong)r->final_minsup};
            (*env)->SetIntArrayRegion(env, sup, 0, n, (const jint*)r->support);
            (*env)->SetDoubleArrayRegion(env, conf, 0, n, r->confidence);
            (*env)->SetLongArrayRegion(env, ao, 0, n + 1, (const jlong*)r->ante_off);
            (*env)->SetLongArrayRegion(env, co, 0, n + 1, (const jlong*)r->cons_off);
            (*env)->SetIntArrayRegion(env, a, 0, na, (const jint*)r->ante);
            (*env)->SetIntArrayRegion(env, c, 0, nc, (const jint*)r->cons);
            (*env)->SetLongArrayRegion(env, meta, 0, 2, m);
            res = (*env)->NewObjectArray(env, 7, obj, NULL);
            if (res) {
                jobject parts[7] = {sup, conf, ao, a, co, c, meta};
                for (int i = 0; i < 7; ++i) (*env)->SetObjectArrayElement(env, res, i, parts[i]);
            }
        } else {
            throw_exception(env, "result copy", FSM_ENOMEM, "JVM array allocation failed");
        }
        fsm_rules_free(r);
    }
    fsm_db_free(db);
    release_ctx(ctx, &dl, rc);
    return res;
}
