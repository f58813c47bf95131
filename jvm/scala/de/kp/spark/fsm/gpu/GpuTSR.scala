package de.kp.spark.fsm.gpu

import org.apache.spark.rdd.RDD

/**
 * Drop-in body for TSR.extractRDDRules
 * (/root/reference/src/main/scala/de/kp/spark/fsm/TSR.scala:31), same
 * signature.  Replaces the item-range job, the Vertical aggregate, the
 * sequences collect and the driver-side TopSeqRules run (TSR.scala:41-105):
 * libfsm parses the records with TSR.newSequence's rules (TSR.scala:109-143),
 * builds the vertical DB and sid bitmaps in HBM and counts every expansion on
 * the GPU, replaying the top-k order on the host.  Sequence ids must be dense
 * 0..N-1 in record order, as the reference requires (TSR.scala:95,103).
 * TSRActor.train (TSRActor.scala:53-62) stays unchanged.
 */
object GpuTSR {

  def extractRDDRules(dataset: RDD[(Int, String)], k: Int, minconf: Double): List[GpuRule] = {
    val recs = dataset.collect()
    val res = FsmNative.tsr(recs.map(_._1), recs.map(_._2), k, minconf, FsmNative.devices)
    val sup = res(0).asInstanceOf[Array[Int]]
    val conf = res(1).asInstanceOf[Array[Double]]
    val anteOff = res(2).asInstanceOf[Array[Long]]
    val ante = res(3).asInstanceOf[Array[Int]]
    val consOff = res(4).asInstanceOf[Array[Long]]
    val cons = res(5).asInstanceOf[Array[Int]]
    (0 until sup.length).map { q =>
      new GpuRule(ante.slice(anteOff(q).toInt, anteOff(q + 1).toInt),
        cons.slice(consOff(q).toInt, consOff(q + 1).toInt), sup(q), conf(q))
    }.toList
  }
}
