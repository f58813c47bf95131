package de.kp.spark.fsm.gpu

/**
 * The result objects the drop-in bodies return.  The reference's element types
 * (de.kp.core.spade.Pattern, de.kp.core.tsr.Rule) live in unvendored modules;
 * their callers use exactly these methods:
 *   Pattern.serialize(): String                    actor/SPADEActor.scala:49
 *   Rule.getItemset1/getItemset2: Array[Int],
 *   getAbsoluteSupport: Int, getConfidence: Double actor/TSRActor.scala:55-59
 * A maintainer either makes these classes extend the reference types or
 * declares the List element type as these traits; SPADEActor and TSRActor
 * compile unchanged either way.
 */
trait SerializablePattern { def serialize(): String }

trait SequentialRule {
  def getItemset1(): Array[Int]
  def getItemset2(): Array[Int]
  def getAbsoluteSupport(): Int
  def getConfidence(): Double
}

/**
 * One frequent sequence.  serialize() renders the SPMF form the actor parses
 * (SPADEActor.scala:49-56): every itemset's items (ascending) then " -1 ",
 * then "| " and the absolute support, e.g. "1 2 -1 3 -1 | 42".
 */
final class GpuPattern(val itemsets: Array[Array[Int]], val support: Int) extends SerializablePattern {
  override def serialize(): String = {
    val sb = new StringBuilder
    for (set <- itemsets) {
      sb.append(set.mkString(" ")).append(" -1 ")
    }
    sb.append("| ").append(support)
    sb.toString
  }
  override def toString: String = serialize()
}

/** One top-k sequential rule X => Y (TSRActor.scala:53-62 reads these four methods). */
final class GpuRule(antecedent: Array[Int], consequent: Array[Int], support: Int, confidence: Double)
    extends SequentialRule {
  override def getItemset1(): Array[Int] = antecedent
  override def getItemset2(): Array[Int] = consequent
  override def getAbsoluteSupport(): Int = support
  override def getConfidence(): Double = confidence
  override def toString: String =
    antecedent.mkString(",") + " ==> " + consequent.mkString(",") + " #SUP: " + support + " #CONF: " + confidence
}
