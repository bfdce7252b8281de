"""Echoes one duplex message back, then sends 'end'."""
from blendtorch import btb

btargs, remainder = btb.parse_blendtorch_args()
duplex = btb.DuplexChannel(btargs.btsockets['CTRL'], btid=btargs.btid, lingerms=5000)
msg = duplex.recv(timeoutms=5000)
duplex.send(echo=msg)
duplex.send(msg='end')
