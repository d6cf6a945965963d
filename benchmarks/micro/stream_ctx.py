"""Host cost of the stream-switching idioms on the step's hot path (µs per call):
``with torch.cuda.stream(s)``, a raw ``torch.cuda.set_stream`` pair, ``torch.cuda.current_stream``,
``Stream.wait_stream``, ``Event.record`` + ``Stream.wait_event``, ``Tensor.record_stream``."""
import time

import torch


def t(fn, n=20000):
    for _ in range(200):
        fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    dev = torch.device("cuda", 0)
    cur = torch.cuda.current_stream(dev)
    s = torch.cuda.Stream(dev, priority=-1)
    ev = torch.cuda.Event()
    x = torch.empty(16, device=dev)

    def ctx():
        with torch.cuda.stream(s):
            pass

    def raw():
        torch.cuda.set_stream(s)
        torch.cuda.set_stream(cur)

    def ws():
        s.wait_stream(cur)

    def rec():
        ev.record(s)
        cur.wait_event(ev)

    res = {"with torch.cuda.stream(s)": t(ctx), "set_stream pair": t(raw),
           "current_stream(dev)": t(lambda: torch.cuda.current_stream(dev)), "wait_stream": t(ws),
           "event record + wait_event": t(rec), "record_stream": t(lambda: x.record_stream(s))}
    torch.cuda.synchronize()
    for k, v in res.items():
        print(f"{k:32s} {v:7.2f} us")


if __name__ == "__main__":
    main()
