"""Graphboard: visualise an executor's dataflow graph (reference
python/graphboard/graph2fig.py:11-32, which renders ``executor.topo_order``
with the graphviz package and serves the figure over HTTP).

graphviz is not a dependency here: ``to_dot`` emits Graphviz DOT text (render
it anywhere with ``dot -Tsvg``), and ``to_html`` lays the DAG out itself
(longest-path layering, barycentric ordering inside a layer) into a
self-contained SVG page, which ``show`` serves with the standard library HTTP
server.

    ht.graphboard.show(executor, port=9997)          # http://127.0.0.1:9997/
    open('g.dot', 'w').write(ht.graphboard.to_dot(executor))
"""
from __future__ import annotations

import html
import threading
from typing import Dict, List

_COLORS = {'PlaceholderOp': '#cfe8ff', 'OptimizerOp': '#ffd8a8', 'comm': '#e5dbff', 'grad': '#f1f3f5',
           'default': '#d3f9d8'}


def _nodes(target, name=None):
    from .ops.executor import find_topo_sort
    if hasattr(target, 'subexecutor'):
        sub = target.subexecutor[name] if name else next(iter(target.subexecutor.values()))
        return list(sub.topo_order)
    if hasattr(target, 'topo_order'):
        return list(target.topo_order)
    return find_topo_sort(list(target))


def _kind(n):
    t = type(n).__name__
    if t in _COLORS:
        return t
    if 'Communicate' in t or 'AllToAll' in t or 'Pipeline' in t or 'ParameterServer' in t:
        return 'comm'
    if 'Grad' in t:
        return 'grad'
    return 'default'


def _label(n):
    t = type(n).__name__
    name = getattr(n, 'name', '') or ''
    return '%s\\n%s' % (name, t) if name and name != t else t


def to_dot(target, name=None) -> str:
    nodes = _nodes(target, name)
    ids = {n: i for i, n in enumerate(nodes)}
    lines = ['digraph hetu {', '  rankdir=TB; node [shape=box, style="rounded,filled", fontsize=10];']
    for n, i in ids.items():
        lines.append('  n%d [label="%s", fillcolor="%s"];' % (i, _label(n).replace('"', "'"), _COLORS[_kind(n)]))
    for n, i in ids.items():
        for x in n.inputs:
            if x in ids:
                lines.append('  n%d -> n%d;' % (ids[x], i))
    lines.append('}')
    return '\n'.join(lines)


def layout(nodes) -> Dict[object, tuple]:
    """Layered DAG layout: layer = longest path from a source; order inside a
    layer by the mean position of the inputs (two sweeps)."""
    layer = {}
    for n in nodes:   # topological order
        ins = [x for x in n.inputs if x in layer]
        layer[n] = 1 + max((layer[x] for x in ins), default=-1)
    layers: Dict[int, List] = {}
    for n in nodes:
        layers.setdefault(layer[n], []).append(n)
    pos = {}
    for L in sorted(layers):
        row = layers[L]
        if L > 0:
            def bary(n):
                xs = [pos[x][0] for x in n.inputs if x in pos]
                return sum(xs) / len(xs) if xs else 0.0
            row.sort(key=bary)
        for k, n in enumerate(row):
            pos[n] = (k, L)
    return pos


def to_html(target, name=None, title='hetu graph') -> str:
    nodes = _nodes(target, name)
    pos = layout(nodes)
    W, H, GX, GY = 150, 34, 20, 40
    width = (max((p[0] for p in pos.values()), default=0) + 1) * (W + GX) + GX
    height = (max((p[1] for p in pos.values()), default=0) + 1) * (H + GY) + GY
    xy = {n: (GX + p[0] * (W + GX), GY + p[1] * (H + GY)) for n, p in pos.items()}
    parts = ['<svg xmlns="http://www.w3.org/2000/svg" width="%d" height="%d" font-family="monospace" '
             'font-size="10">' % (width, height),
             '<defs><marker id="a" markerWidth="8" markerHeight="8" refX="6" refY="3" orient="auto">'
             '<path d="M0,0 L0,6 L6,3 z" fill="#868e96"/></marker></defs>']
    for n in nodes:
        x1, y1 = xy[n]
        for s in n.inputs:
            if s in xy:
                x0, y0 = xy[s]
                parts.append('<line x1="%d" y1="%d" x2="%d" y2="%d" stroke="#adb5bd" marker-end="url(#a)"/>'
                             % (x0 + W // 2, y0 + H, x1 + W // 2, y1))
    for n in nodes:
        x, y = xy[n]
        lab = _label(n).split('\\n')
        parts.append('<g><title>%s</title><rect x="%d" y="%d" width="%d" height="%d" rx="6" fill="%s" '
                     'stroke="#495057"/>' % (html.escape(repr(n)), x, y, W, H, _COLORS[_kind(n)]))
        for k, t in enumerate(lab[:2]):
            parts.append('<text x="%d" y="%d" text-anchor="middle">%s</text>'
                         % (x + W // 2, y + 13 + 12 * k, html.escape(t[:24])))
        parts.append('</g>')
    parts.append('</svg>')
    return ('<!doctype html><html><head><meta charset="utf-8"><title>%s</title></head><body>'
            '<h3>%s: %d nodes</h3>%s</body></html>' % (html.escape(title), html.escape(title), len(nodes),
                                                       ''.join(parts)))


def show(target, port=9997, name=None, block=False):
    """Serve the graph page at http://127.0.0.1:port/ (and the DOT at /graph.dot)."""
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
    page = to_html(target, name).encode()
    dot = to_dot(target, name).encode()

    class H(BaseHTTPRequestHandler):
        def do_GET(self):
            body, ctype = (dot, 'text/vnd.graphviz') if self.path.endswith('.dot') else (page, 'text/html')
            self.send_response(200)
            self.send_header('Content-Type', ctype)
            self.send_header('Content-Length', str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    srv = ThreadingHTTPServer(('127.0.0.1', port), H)
    if block:
        srv.serve_forever()
    else:
        threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv
