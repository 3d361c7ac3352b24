// An Akka (classic) actor that drives an mxar job through the master's control bridge
// (docs/BRIDGE.md): the round loop of the reference's AllreduceMaster
// (src/main/scala/sample/cluster/allreduce/AllreduceMaster.scala:58-67,91-97), with the
// workers running natively on the GPUs.
//
// Not compiled in this repository (the build image has no JVM); it only needs Akka 2.5 and
// the JDK. Start the engine with `mxar master 2551 P N C --bridge 2600 --external-rounds`
// plus P workers, then run this actor with host "127.0.0.1", port 2600.
package sample.cluster.allreduce.bridge

import java.io.{BufferedReader, InputStreamReader, PrintWriter}
import java.net.Socket

import akka.actor.{Actor, ActorLogging, Props}

object BridgeDriver {
  final case class Line(json: String)
  def props(host: String, port: Int, maxRound: Int): Props = Props(new BridgeDriver(host, port, maxRound))

  // The bridge's lines are flat JSON objects; a regex per field is enough here.
  private def field(json: String, name: String): Option[String] =
    ("\"" + name + "\"\\s*:\\s*\"?([^\",}]*)").r.findFirstMatchIn(json).map(_.group(1))
}

class BridgeDriver(host: String, port: Int, maxRound: Int) extends Actor with ActorLogging {
  import BridgeDriver._

  private val socket = new Socket(host, port)
  socket.setTcpNoDelay(true)
  private val out = new PrintWriter(socket.getOutputStream, true)
  private val in = new BufferedReader(new InputStreamReader(socket.getInputStream))

  // Reader thread: every bridge line becomes a message to this actor.
  private val reader = new Thread(new Runnable {
    def run(): Unit = {
      var l = in.readLine()
      while (l != null) { self ! Line(l); l = in.readLine() }
    }
  })
  reader.setDaemon(true)
  reader.start()

  private var lastSent = -1  // newest StartAllreduce sent (at most one queued behind the round in flight)

  private def startAllreduce(r: Int): Unit = {  // AllreduceMaster.scala:91-97
    lastSent = r
    log.info(s"----Start allreduce round $r")
    out.println(s"""{"type":"StartAllreduce","round":$r}""")
  }

  def receive: Receive = {
    case Line(json) =>
      field(json, "type") match {
        case Some("InitWorkers") =>
          log.info(s"----workers initialised: $json")
          if (lastSent < 0) startAllreduce(field(json, "startRound").map(_.toInt).getOrElse(0))
        case Some("Accepted") =>
          // round r is running: queue r + 1 now, so the master starts it at r's barrier
          // without waiting for this actor (docs/BRIDGE.md "Queued starts")
          val r = field(json, "round").map(_.toInt).getOrElse(-1)
          if (r == lastSent && r < maxRound) startAllreduce(r + 1)
        case Some("CompleteAllreduce") =>  // AllreduceMaster.scala:58-61
          log.info(s"----Node ${field(json, "srcId").getOrElse("?")} completes allreduce round ${field(json, "round").getOrElse("?")}")
        case Some("RoundComplete") =>  // the barrier of AllreduceMaster.scala:62-66
          log.info(s"----round ${field(json, "round").getOrElse("?")} complete")
        case Some("AllreduceFinished") =>
          log.info("----All rounds complete"); context.stop(self)
        case Some("Error") => log.warning(s"bridge refused: $json")
        case _ =>
      }
  }

  override def postStop(): Unit = socket.close()
}
