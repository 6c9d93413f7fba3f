"""Client operation history (history.go, operation.go) of simulated ABD runs.

`History` mirrors the reference type: operations sharded by key
(`Add`/`AddOperation`, history.go:31-52), `WriteFile` (history.go:74-113, the
"history.csv" the benchmark writes at benchmark.go:187) and `ReadFile`
(history.go:116-178, the 5-column log that checker/checker.go reads).  It is
filled from the device's recorded ops (`paxisim_history`): a write has
input = value and output = nil, a read input = nil and output = value, as the
benchmark worker records them (benchmark.go:253-273).

Times are virtual steps; `step_ns` maps a step to the nanosecond timestamps
the reference uses (op.start/op.end are ns since the benchmark start).
Linearizability of a simulated history is checked on the device over the whole
handle (`Simulation.linearizable`, checker.go:69-104); this module is the
export/import side only.
"""
import csv


class Operation:
    """operation.go:5-11: input, output (None = nil) and start/end timestamps (ns)."""
    __slots__ = ("input", "output", "start", "end")

    def __init__(self, input, output, start, end):
        self.input, self.output, self.start, self.end = input, output, start, end

    def __eq__(self, o):   # operation.equal (operation.go:21-23)
        return (self.input, self.output, self.start, self.end) == (o.input, o.output, o.start, o.end)

    def __repr__(self):
        return f"Operation({self.input!r}, {self.output!r}, {self.start}, {self.end})"


def _v(x):
    """Go's %v of an interface{}: <nil> for nil, decimal for ints, the string itself."""
    return "<nil>" if x is None else str(x)


class History:
    def __init__(self):
        self.shard = {}          # key -> [Operation]
        self.operations = []

    def add(self, key, input, output, start, end):          # History.Add (history.go:31-41)
        self.add_operation(key, Operation(input, output, start, end))

    def add_operation(self, key, op):                      # History.AddOperation (history.go:44-52)
        self.shard.setdefault(key, []).append(op)
        self.operations.append(op)

    @classmethod
    def from_simulation(cls, sim, clusters=None, step_ns=1_000_000):
        """Histories of `clusters` (default: all) of an ABD Simulation, one
        History per cluster, in the device's canonical order."""
        if clusters is None:
            clusters = range(sim.cfg.clusters)
        out = []
        for c in clusters:
            h = cls()
            for key, is_write, value, start, end in sim.history(c):
                if is_write:
                    h.add(key, value, None, start * step_ns, end * step_ns)
                else:
                    h.add(key, None, value, start * step_ns, end * step_ns)
            out.append(h)
        return out

    def write_file(self, path):
        """History.WriteFile (history.go:74-113): `path`.csv with
        "input,output,start,end" (seconds, %f) in start order, and a
        "PerSecond <mean latency ms> <ops>" line each time an op ends past the
        next whole second."""
        self.operations.sort(key=lambda o: o.start)   # sort.Sort(byTime) (operation.go:30-34)
        lines = []
        latency, throughput, s = 0.0, 0, 1.0
        for o in self.operations:
            start, end = o.start / 1e9, o.end / 1e9
            lines.append("%s,%s,%f,%f\n" % (_v(o.input), _v(o.output), start, end))
            latency += end - start
            throughput += 1
            if end > s:
                lines.append("PerSecond %f %d\n" % (latency / throughput * 1000.0, throughput))
                latency, throughput = 0.0, 0
                s += 1
        with open(path + ".csv", "w") as f:
            f.writelines(lines)

    def write_log(self, path):
        """The 5-column "key,input,output,start,end" log (ns) that ReadFile
        parses (history.go:133-175), nil written as "null"."""
        with open(path, "w", newline="") as f:
            w = csv.writer(f, lineterminator="\n")
            for key in sorted(self.shard):
                for o in self.shard[key]:
                    w.writerow([key, "null" if o.input is None else o.input,
                                "null" if o.output is None else o.output, o.start, o.end])

    @classmethod
    def read_file(cls, path):
        """History.ReadFile (history.go:116-178): values stay strings as in Go;
        "null" or "" is nil; fewer than 5 columns is a format error."""
        h = cls()
        with open(path, newline="") as f:
            for rec in csv.reader(f):
                if len(rec) < 5:
                    raise ValueError("operation history file format error")
                key = int(rec[0])
                inp = None if rec[1] in ("null", "") else rec[1]
                out = None if rec[2] in ("null", "") else rec[2]
                h.add_operation(key, Operation(inp, out, int(rec[3]), int(rec[4])))
        return h
