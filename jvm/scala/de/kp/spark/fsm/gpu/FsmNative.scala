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
      loaded = try {
        System.loadLibrary("fsm_jni")
        // the idle contexts the shim keeps between requests go with the JVM
        Runtime.getRuntime.addShutdownHook(new Thread(new Runnable { def run(): Unit = FsmNativeJNI.release() }))
        None
      } catch { case t: Throwable => Some(t) }
    }
    loaded match {
      case Some(t) => throw new Exception("libfsm_jni could not be loaded: " + t.getMessage, t)
      case None =>
    }
  }

  /** The first GPU device of this JVM's requests: -Dfsm.device=N (default 0). */
  def device: Int = Integer.getInteger("fsm.device", 0)

  /**
   * The GPUs one request shards over (SURVEY §8(b): 1, 2, 4 or 8), from -Dfsm.devices:
   *   absent or "1"  -> Array(device)                   one GPU
   *   "N"            -> device, device+1, ..., device+N-1
   *   "0,1,2,3"      -> exactly these ordinals (one may repeat: several ranks on one GPU)
   * A malformed value surfaces as java.lang.Exception from the call (TrainActor.scala:66).
   */
  def devices: Array[Int] = {
    val v = System.getProperty("fsm.devices", "").trim
    try {
      if (v.isEmpty) Array(device)
      else if (v.contains(",")) v.split(",").map(_.trim.toInt)
      else (0 until math.max(1, v.toInt)).map(device + _).toArray
    } catch {
      case e: NumberFormatException => throw new Exception("bad -Dfsm.devices value: " + v, e)
    }
  }

  def spade(sids: Array[Int], lines: Array[String], support: Double, dfs: Boolean,
            devices: Array[Int]): Array[AnyRef] = {
    ensureLoaded()
    FsmNativeJNI.spade(sids, lines, support, dfs, devices)
  }

  def tsr(sids: Array[Int], lines: Array[String], k: Int, minconf: Double, devices: Array[Int]): Array[AnyRef] = {
    ensureLoaded()
    FsmNativeJNI.tsr(sids, lines, k, minconf, devices)
  }
}
