"""Protocol messages and user I/O records (same names, fields and field order as the
reference's `AllreduceMessage.scala:7-20` and `DataWrapper.scala:3-7`).

All classes are native (C++) types so that messages cross the actor runtime without
Python overhead; payload fields accept any float sequence / numpy array (host) or a
torch tensor on the GPU (device payloads: the HIP device plane in
`csrc/hip/device_plane.hip`; tensor dataSources for the round engine: `engine.PlaneJob`).
"""
from ._native import C

InitWorkers = C.InitWorkers
StartAllreduce = C.StartAllreduce
ScatterBlock = C.ScatterBlock
ReduceBlock = C.ReduceBlock
CompleteAllreduce = C.CompleteAllreduce
AllReduceInputRequest = C.AllReduceInputRequest
AllReduceInput = C.AllReduceInput
AllReduceOutput = C.AllReduceOutput
MemberUp = C.MemberUp
Terminated = C.Terminated
AllreduceFinished = C.AllreduceFinished
PoisonPill = C.PoisonPill
TextMessage = C.TextMessage
ActorRef = C.ActorRef
# extensions: the master's typed round deadline, and a plane's round completion (local only)
RoundTimeout = C.RoundTimeout
PlaneRoundDone = C.PlaneRoundDone

__all__ = [
    "InitWorkers", "StartAllreduce", "ScatterBlock", "ReduceBlock", "CompleteAllreduce",
    "AllReduceInputRequest", "AllReduceInput", "AllReduceOutput", "MemberUp", "Terminated",
    "AllreduceFinished", "PoisonPill", "TextMessage", "ActorRef", "RoundTimeout", "PlaneRoundDone",
]
