"""A rendezvous port for the multi-process tests.

bind(0) hands out a port of the kernel's ephemeral range, the range every outgoing
connection on the box draws from too, so between this probe and the rank-0 store
binding it another process can take it (EADDRINUSE, seen once on a shared GPU box).
The port is drawn instead from below that range, at random, and checked free."""
import random
import socket


def free_port() -> int:
    lo = 20000
    try:  # the ephemeral range's start (32768 by default)
        hi = int(open("/proc/sys/net/ipv4/ip_local_port_range").read().split()[0])
    except (OSError, ValueError, IndexError):
        hi = 32768
    hi = max(hi, lo + 1000)
    rng = random.SystemRandom()
    for _ in range(200):
        p = rng.randrange(lo, hi)
        s = socket.socket()
        try:
            s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    s = socket.socket()  # (every probe taken: fall back to an ephemeral one)
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p
