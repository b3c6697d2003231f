"""``paddle.distributed.utils`` (reference: python/paddle/distributed/utils.py): the MoE
all-to-all exchanges ``global_scatter`` / ``global_gather`` and host helpers."""
import socket

from ..incubate.distributed.models.moe.utils import global_scatter, global_gather  # noqa: F401

__all__ = ["global_scatter", "global_gather", "get_host_name_ip", "find_free_ports"]


def get_host_name_ip():
    try:
        name = socket.gethostname()
        return name, socket.gethostbyname(name)
    except OSError:
        return None


def find_free_ports(num):
    ports, socks = set(), []
    for _ in range(num):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        ports.add(s.getsockname()[1])
        socks.append(s)
    for s in socks:
        s.close()
    return ports
