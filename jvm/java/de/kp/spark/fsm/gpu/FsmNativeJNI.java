package de.kp.spark.fsm.gpu;

/**
 * Static JNI declarations bound by jvm/native/fsm_jni.c
 * (Java_de_kp_spark_fsm_gpu_FsmNativeJNI_spade / _tsr).  Declared in Java so
 * the symbols are plain static methods (a Scala object's natives would bind as
 * instance methods of FsmNative$).  Callers go through FsmNative.scala, which
 * loads the library and turns load failures into java.lang.Exception.
 */
public final class FsmNativeJNI {
    private FsmNativeJNI() {}

    /** [support int[], patOff long[], setOff long[], items int[], {total, minsup} long[]].
     *  devices: the HIP ordinals of the mine's ranks (one: a single GPU; more: one call sharded
     *  over in-process ranks, rank r on devices[r]). */
    public static native Object[] spade(int[] sids, String[] lines, double support, boolean dfs, int[] devices);

    /** [support int[], confidence double[], anteOff long[], ante int[], consOff long[], cons int[],
     *  {total, finalMinsup} long[]] */
    public static native Object[] tsr(int[] sids, String[] lines, int k, double minconf, int[] devices);

    /** Destroys the contexts kept idle between requests (fsm_jni.c keeps up to 4, keyed by device
     *  list, so a request does not rebuild its rank group); FsmNative registers it at JVM shutdown. */
    public static native void release();
}
