"""Small networking helpers (reference: pkg_pytorch/blendtorch/btt/utils.py:2-17)."""
import socket


def get_primary_ip():
    """IPv4 address of the interface holding the default route, else 127.0.0.1.

    A UDP socket is "connected" to an unroutable address; no packet is sent,
    but the kernel picks the outgoing interface, whose address we read back.
    """
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        s.connect(('10.255.255.255', 1))
        ip = s.getsockname()[0]
    except OSError:
        ip = '127.0.0.1'
    finally:
        s.close()
    return ip
