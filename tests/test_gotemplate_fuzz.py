"""Mutation fuzz of the Go text/template engine (utils/gotemplate*.py).

Seeds are the packaged templates (assets/templates, the ones
reference/internal/assets/templates renders) plus small templates that reach
every action, builtin and verb.  Each seed is mutated with template tokens and
run against random data.  What Go guarantees is checked: parsing or
executing returns a result or a template error and never anything else, and
the interpreted run and the compiled run (``M2K_TEMPLATE_COMPILE_AFTER``) give
the same text."""

import os
import random

import pytest

from move2kube_amd import assets
from move2kube_amd.utils.gotemplate import Template, TemplateError

SMALL = [
    '{{if eq .port 8080.0}}EXPOSE {{.port}}{{end}}',
    '{{range $i, $v := .L}}{{$i}}={{$v}},{{end}}',
    '{{with .M}}{{.k}}{{else}}none{{end}}',
    '{{printf "%5.2f|%-5d|%q" .f .n .s}}',
    '{{index .M "k"}} {{len .L}} {{slice .s 1 2}}',
    '{{define "t"}}[{{.}}]{{end}}{{template "t" .s}}{{block "b" .}}x{{end}}',
    '{{$x := 1}}{{$x = 2}}{{$x}}',
    '{{and .a .b}} {{or .a .b}} {{not .a}} {{html "<>"}} {{js "\'"}} {{urlquery "a b"}} {{print 1 2}} {{println "x"}}',
    '{{- .s -}} {{/* c */}} {{.M.k.z}} {{(.M).k}} {{call .s}} {{lt 1 2}} {{le 1.0 .f}} {{ne .s "x"}}',
    '{{printf "%[2]*[1]d %x %X %o %b %c %U %e %g %s %v %+v %#v %T %p" 12 5 .f .L .M .s .n}}',
]
TOKENS = ["{{", "}}", "(", ")", "|", ".", "$", "$x", ":=", "=", " ", "if", "else", "end", "range", "with", "define",
          "template", "block", '"', "'", "`", "1", "1.5", "0x1f", "nil", "true", ".L", ".M", ".s", "eq", "printf",
          "index", "len", "slice", "call", "-", "\n", "%", "%v", "%d", "%!", "\\", "%[9]d", "%*d", "1e308", "-0",
          "0b1", "'a'", "1i"]


def _seeds():
    out = list(SMALL)
    for name in sorted(os.listdir(assets.TEMPLATES_DIR)):
        with open(os.path.join(assets.TEMPLATES_DIR, name), encoding="utf-8") as f:
            out.append(f.read())
    return out


def _data(rnd, d=0):
    c = rnd.randint(0, 7 if d < 3 else 5)
    if c == 6:
        return [_data(rnd, d + 1) for _ in range(rnd.randint(0, 3))]
    if c == 7:
        return {k: _data(rnd, d + 1) for k in rnd.sample(["k", "z", "a", "b"], rnd.randint(0, 3))}
    return [None, True, 1.5, 8080.0, "abc", "<é>"][c]


def _mutate(rnd, src):
    s = list(src)
    for _ in range(rnd.randint(1, 5)):
        i = rnd.randrange(len(s) + 1)
        op = rnd.randint(0, 2)
        if op == 0 and i < len(s):
            del s[i]
        elif op == 1:
            s[i:i] = list(rnd.choice(TOKENS))
        elif i < len(s):
            s[i] = rnd.choice(TOKENS)
    return "".join(s)


@pytest.mark.parametrize("seed", range(4))
def test_mutated_templates_fail_only_as_template_errors(seed):
    rnd = random.Random(seed)
    seeds = _seeds()
    executed = 0
    for _ in range(1500):
        src = _mutate(rnd, rnd.choice(seeds))
        data = {"port": 8080.0, "L": _data(rnd), "M": _data(rnd), "s": rnd.choice(["abc", "", "é", None]),
                "f": rnd.choice([1.5, None, "x"]), "n": rnd.choice([3, 3.0, "3", None]), "a": _data(rnd), "b": _data(rnd)}
        try:
            t = Template(src)
            first = t.execute(data)     # interpreted
            second = t.execute(data)    # compiled (COMPILE_AFTER=1)
        except TemplateError:
            continue
        assert isinstance(first, str)
        assert first == second, src
        executed += 1
    assert executed > 100     # the mutations leave plenty of templates that run
