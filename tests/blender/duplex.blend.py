"""Scene script for tests/test_duplex.py: answer the first message on the CTRL
channel with an echo of it, then say 'end'. A 5 s linger lets both replies
leave before Blender exits."""
from blendtorch import btb

btargs, _ = btb.parse_blendtorch_args()
channel = btb.DuplexChannel(btargs.btsockets['CTRL'], btid=btargs.btid, lingerms=5000)
request = channel.recv(timeoutms=5000)
for reply in ({'echo': request}, {'msg': 'end'}):
    channel.send(**reply)
