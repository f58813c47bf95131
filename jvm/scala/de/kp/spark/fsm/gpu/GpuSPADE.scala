package de.kp.spark.fsm.gpu

import org.apache.spark.rdd.RDD

/**
 * Drop-in body for SPADE.extractRDDPatterns
 * (/root/reference/src/main/scala/de/kp/spark/fsm/SPADE.scala:36), same
 * signature.  The reference parses every record twice, builds the F1 id-lists
 * in one Spark task and mines on the driver thread (SPADE.scala:45-138); here
 * the records are collected once and handed to libfsm, which parses them with
 * the same rules (SPADE.scala:145-212), flattens them into HBM and mines on the
 * GPU.  A maintainer replaces the body of SPADE.extractRDDPatterns with
 *   GpuSPADE.extractRDDPatterns(dataset, support, dfs, stats)
 * and SPADEActor.train (SPADEActor.scala:47-58) stays byte-for-byte unchanged.
 */
object GpuSPADE {

  def extractRDDPatterns(dataset: RDD[(Int, String)], support: Double, dfs: Boolean = true,
                         stats: Boolean = true): List[GpuPattern] = {
    val recs = dataset.collect()
    val res = FsmNative.spade(recs.map(_._1), recs.map(_._2), support, dfs, FsmNative.devices)
    val sup = res(0).asInstanceOf[Array[Int]]
    val patOff = res(1).asInstanceOf[Array[Long]]
    val setOff = res(2).asInstanceOf[Array[Long]]
    val items = res(3).asInstanceOf[Array[Int]]
    if (stats) {
      // replaces algorithm.printStatistics() (SPADE.scala:136)
      val meta = res(4).asInstanceOf[Array[Long]]
      println("GPU SPADE: " + sup.length + " frequent sequences, " + meta(0) + " sequences, minsup " + meta(1))
    }
    (0 until sup.length).map { p =>
      val sets = (patOff(p).toInt until patOff(p + 1).toInt).map { s =>
        items.slice(setOff(s).toInt, setOff(s + 1).toInt)
      }.toArray
      new GpuPattern(sets, sup(p))
    }.toList
  }
}
