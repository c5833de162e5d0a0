"""Reader for the AMPL-style ``.dat`` subset the reference's UC data uses.

The reference loads ``RootNode.dat`` + ``NodeN.dat`` with Pyomo's ``DataPortal``
(paperruns/larger_uc/uc_funcs.py:32-34).  Pyomo is not in this image, so this module
reads the statement forms those files hold (paperruns/larger_uc/RootNode.dat,
1000scenarios_wind/Node*.dat):

    param NAME := value ;                       scalar
    param NAME := <index...> value  (per line)  indexed
    param: C1 C2 ... := <index...> v1 v2 ...    tabular, one row per line
    set NAME := e1 e2 ... ;
    set NAME[idx] := e1 e2 ... ;

``#`` starts a comment.  Numbers become ``int`` when they are integer literals and
``float`` otherwise, as Pyomo's data parser does; other tokens stay strings.
"""


def _atom(tok):
    try:
        return int(tok)
    except ValueError:
        pass
    try:
        return float(tok)
    except ValueError:
        return tok


def _key(toks):
    return _atom(toks[0]) if len(toks) == 1 else tuple(_atom(t) for t in toks)


def parse_dat(text, params=None, sets=None):
    """Parse ``text``; returns ``(params, sets)`` dicts, updating the given ones
    (a later file overrides entries of an earlier one, as successive
    ``DataPortal.load`` calls do).  An indexed param is a dict key -> value; a
    tabular ``param:`` statement fills one such dict per column."""
    params = {} if params is None else params
    sets = {} if sets is None else sets
    lines = [ln.split("#", 1)[0] for ln in text.splitlines()]
    body = "\n".join(lines)
    for stmt in body.split(";"):
        stmt = stmt.strip()
        if not stmt:
            continue
        if ":=" not in stmt:
            raise ValueError(f"unsupported .dat statement: {stmt[:60]!r}")
        head, rest = stmt.split(":=", 1)
        head = head.split()
        kind = head[0]
        if kind == "set":
            name = " ".join(head[1:])
            sets[name] = [_atom(t) for t in rest.split()]
        elif kind == "param:":
            cols = head[1:]
            for c in cols:
                params.setdefault(c, {})
            for ln in rest.splitlines():
                toks = ln.split()
                if not toks:
                    continue
                k = len(toks) - len(cols)
                if k < 1:
                    raise ValueError(f"tabular row too short: {ln!r}")
                key = _key(toks[:k])
                for c, v in zip(cols, toks[k:]):
                    params[c][key] = _atom(v)
        elif kind == "param":
            if len(head) != 2:
                raise ValueError(f"unsupported param header: {' '.join(head)!r}")
            name = head[1]
            rows = [ln.split() for ln in rest.splitlines() if ln.split()]
            if len(rows) == 1 and len(rows[0]) == 1:
                params[name] = _atom(rows[0][0])
            else:
                d = params.get(name)
                if not isinstance(d, dict):
                    d = {}
                for toks in rows:
                    d[_key(toks[:-1])] = _atom(toks[-1])
                params[name] = d
        else:
            raise ValueError(f"unsupported .dat statement kind {kind!r}")
    return params, sets


def load_dat(path, params=None, sets=None):
    with open(path) as f:
        return parse_dat(f.read(), params, sets)


def dump_data(params, sets):
    """JSON-able form of (params, sets): indexed params as [[key, value], ...] with tuple
    keys as lists (load_data inverts it exactly)."""
    P = {}
    for k, v in params.items():
        if isinstance(v, dict):
            P[k] = {"indexed": [[list(kk) if isinstance(kk, tuple) else kk, vv] for kk, vv in v.items()]}
        else:
            P[k] = {"scalar": v}
    return {"params": P, "sets": sets}


def load_data(obj):
    """Inverse of dump_data."""
    params = {}
    for k, v in obj["params"].items():
        if "scalar" in v:
            params[k] = v["scalar"]
        else:
            params[k] = {(tuple(kk) if isinstance(kk, list) else kk): vv for kk, vv in v["indexed"]}
    return params, {k: list(v) for k, v in obj["sets"].items()}
