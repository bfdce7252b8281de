"""Publishes its parsed launch arguments (mirrors the reference test script's role)."""
from blendtorch import btb

btargs, remainder = btb.parse_blendtorch_args()
# linger so the message is flushed before the interpreter exits
pub = btb.DataPublisher(btargs.btsockets['DATA'], btargs.btid, lingerms=10000)
pub.publish(btargs=vars(btargs), remainder=remainder)
