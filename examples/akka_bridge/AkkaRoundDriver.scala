// An unmodified Akka 2.5 actor (classic remoting, Java serialization - the reference's own
// stack) that drives an mxar job over akka.tcp (docs/AKKA_WIRE.md): the round loop of the
// reference's AllreduceMaster (AllreduceMaster.scala:58-67,91-97), with the workers running
// natively on the GPUs. Unlike BridgeDriver.scala it needs no socket code: the master's
// endpoint speaks akka.tcp and takes the reference's own message classes.
//
// Not compiled in this repository (the build image has no JVM). It needs Akka 2.5 with
// `akka.actor.provider = remote` and the reference's messages (AllreduceMessage.scala) on the
// classpath. Start the engine with `mxar master 2551 P N C --akka-port 2600 --external-rounds`
// plus P workers, then run this actor with master address
// "akka.tcp://ClusterSystem@127.0.0.1:2600". If the engine reports a serialVersionUID
// mismatch, pass the values `serialver` prints for StartAllreduce / CompleteAllreduce to the
// master (`--akka-suid-start`, `--akka-suid-complete`).
package sample.cluster.allreduce.driver

import scala.concurrent.duration._

import akka.actor.{Actor, ActorIdentity, ActorLogging, ActorRef, Identify, Props, ReceiveTimeout}
import sample.cluster.allreduce.{CompleteAllreduce, StartAllreduce}

object AkkaRoundDriver {
  def props(masterAddress: String, workers: Int, maxRound: Int, thAllreduce: Float = 1f): Props =
    Props(new AkkaRoundDriver(masterAddress, workers, maxRound, thAllreduce))
}

class AkkaRoundDriver(masterAddress: String, workers: Int, maxRound: Int, thAllreduce: Float)
    extends Actor with ActorLogging {
  private val selection = context.actorSelection(s"$masterAddress/user/master")
  private var round = 0
  private var numComplete = 0

  override def preStart(): Unit = {
    selection ! Identify("mxar-master")
    context.setReceiveTimeout(3.seconds)
  }

  def receive: Receive = {
    case ActorIdentity(_, Some(master)) =>
      context.setReceiveTimeout(2.seconds)  // re-sends a start the master refused (below)
      log.info(s"----master resolved: $master")
      context.become(driving(master))
      master ! StartAllreduce(round)
    case ActorIdentity(_, None) | ReceiveTimeout =>
      selection ! Identify("mxar-master")  // the engine is not up yet
  }

  // AllreduceMaster.scala:58-67: count completions of the current round, start the next
  // one at the threshold. A StartAllreduce sent before the workers are initialised is
  // refused by the master (it logs it); the timeout re-sends it.
  private def driving(master: ActorRef): Receive = {
    case c: CompleteAllreduce =>
      if (c.round == round) {
        numComplete += 1
        if (numComplete >= workers * thAllreduce) {
          log.info(s"----$numComplete (out of $workers) workers complete round $round")
          if (round < maxRound) {
            round += 1
            numComplete = 0
            master ! StartAllreduce(round)
          } else {
            log.info(s"----finished ${maxRound + 1} rounds")
            context.stop(self)
          }
        }
      }
    case ReceiveTimeout => master ! StartAllreduce(round)
  }
}
