package de.kp.spark.fsm.gpu

/**
 * Loader and entry points of libfsm_jni.so (jvm/native/fsm_jni.c, bound through
 * FsmNativeJNI.java) over libfsm.so
 * (include/fsm.h).  Loading failures surface as java.lang.Exception, never as
 * UnsatisfiedLinkError: TrainActor only catches Exception
 * (actor/TrainActor.scala:66), and an Error would leave the request's status
 * at MINING_STARTED.
 *
 * The arrays returned are the C ABI's result CSR, unchanged:
 *   spade -> [support: Array[Int], patOff: Array[Long], setOff: Array[Long],
 *             items: Array[Int], meta: Array[Long](total, minsup)]
 *   tsr   -> [support: Array[Int], confidence: Array[Double], anteOff: Array[Long],
 *             ante: Array[Int], consOff: Array[Long], cons: Array[Int],
 *             meta: Array[Long](total, finalMinsup)]
 */
object FsmNative {

  @volatile private var loaded: Option[Throwable] = null

  /** System.loadLibrary("fsm_jni") once; a failure is kept and rethrown as Exception on every call. */
  private def ensureLoaded(): Unit = synchronized {
    if (loaded == null) {
      loaded = try { System.loadLibrary("fsm_jni"); None } catch { case t: Throwable => Some(t) }
    }
    loaded match {
      case Some(t) => throw new Exception("libfsm_jni could not be loaded: " + t.getMessage, t)
      case None =>
    }
  }

  /** The GPU device of this JVM's requests: -Dfsm.device=N (default 0). */
  def device: Int = Integer.getInteger("fsm.device", 0)

  def spade(sids: Array[Int], lines: Array[String], support: Double, device: Int): Array[AnyRef] = {
    ensureLoaded()
    FsmNativeJNI.spade(sids, lines, support, device)
  }

  def tsr(sids: Array[Int], lines: Array[String], k: Int, minconf: Double, device: Int): Array[AnyRef] = {
    ensureLoaded()
    FsmNativeJNI.tsr(sids, lines, k, minconf, device)
  }
}
