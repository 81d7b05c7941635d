"""Which multi-stream fork/join patterns survive HIP graph capture (each variant in a child
process, so a crash in one is reported, not fatal):  python3 tools/probes/capture_probe.py"""
import subprocess
import sys

import torch


def work(x):
    x.mul_(1.0001).add_(1.0)


def variant(name):
    dev = torch.device("cuda:0")
    xs = [torch.ones(1 << 20, device=dev) for _ in range(8)]
    a, w0, w1 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())

    def body():
        s = torch.cuda.current_stream()
        if name == "fork_once":
            a.wait_stream(s)
            work(xs[0])
            with torch.cuda.stream(a):
                work(xs[1])
            s.wait_stream(a)
        elif name == "fork_twice":
            for k in range(2):
                a.wait_stream(s)
                work(xs[0])
                with torch.cuda.stream(a):
                    work(xs[1])
                s.wait_stream(a)
        elif name in ("nested", "nested_twice", "nested_cross"):
            a.wait_stream(s)
            reps = 1 if name == "nested" else 2
            for k in range(reps):
                # lane 0 (s) with side w0
                w0.wait_stream(s)
                with torch.cuda.stream(w0):
                    work(xs[2])
                work(xs[0])
                s.wait_stream(w0)
                e0 = s.record_event()
                with torch.cuda.stream(a):
                    w1.wait_stream(a)
                    with torch.cuda.stream(w1):
                        work(xs[3])
                    work(xs[1])
                    a.wait_stream(w1)
                    e1 = a.record_event()
                if name == "nested_cross":
                    s.wait_event(e1)
                    a.wait_event(e0)
            s.wait_stream(a)
        elif name == "nested_plain":
            a.wait_stream(s)
            with torch.cuda.stream(a):
                w1.wait_stream(a)
                with torch.cuda.stream(w1):
                    work(xs[3])
                work(xs[1])
                a.wait_stream(w1)
            s.wait_stream(a)
        elif name == "prejoined":
            a.wait_stream(s)
            w1.wait_stream(s)
            with torch.cuda.stream(a):
                work(xs[1])
                w1.wait_stream(a)
                with torch.cuda.stream(w1):
                    work(xs[3])
                a.wait_stream(w1)
            s.wait_stream(a)
        elif name == "stray_event":
            a.wait_stream(s)
            work(xs[0])
            e = s.record_event()
            with torch.cuda.stream(a):
                work(xs[1])
            s.wait_stream(a)
        elif name == "prejoined_twice":
            a.wait_stream(s)
            w0.wait_stream(s)
            w1.wait_stream(s)
            for k in range(2):
                w0.wait_stream(s)
                with torch.cuda.stream(w0):
                    work(xs[2])
                s.wait_stream(w0)
                e0 = torch.cuda.Event()
                e0.record(s)
                with torch.cuda.stream(a):
                    work(xs[1])
                    w1.wait_stream(a)
                    with torch.cuda.stream(w1):
                        work(xs[3])
                    a.wait_stream(w1)
                    e1 = torch.cuda.Event()
                    e1.record(a)
                s.wait_event(e1)
                a.wait_event(e0)
            s.wait_stream(a)
        elif name == "nested_cross_events":
            # the model's exact shape: torch.cuda.Event() objects recorded then waited
            a.wait_stream(s)
            for k in range(2):
                w0.wait_stream(s)
                with torch.cuda.stream(w0):
                    work(xs[2])
                s.wait_stream(w0)
                e0 = torch.cuda.Event()
                e0.record(s)
                with torch.cuda.stream(a):
                    w1.wait_stream(a)
                    with torch.cuda.stream(w1):
                        work(xs[3])
                    a.wait_stream(w1)
                    e1 = torch.cuda.Event()
                    e1.record(a)
                s.wait_event(e1)
                a.wait_event(e0)
            s.wait_stream(a)

    with torch.cuda.stream(cap):
        body()          # eager once
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=cap, capture_error_mode="thread_local"):
        body()
    torch.cuda.current_stream().wait_stream(cap)
    g.replay()
    torch.cuda.synchronize()
    print(name, "ok", float(xs[0][0]))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--one":
        variant(sys.argv[2])
        sys.exit(0)
    for v in sys.argv[1:] or ["nested_plain", "prejoined", "stray_event", "prejoined_twice"]:
        r = subprocess.run([sys.executable, __file__, "--one", v], capture_output=True, text=True, timeout=120)
        print(v, "rc", r.returncode, r.stdout.strip()[-200:], r.stderr.strip()[-300:] if r.returncode else "")
