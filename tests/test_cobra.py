"""Command-line parsing and texts as cobra v1.1.1 / pflag v1.0.5 produce them
for the reference's command tree (``cmd/move2kube/*.go``; ``go.mod:30``):
help and usage templates, ``FlagUsages`` columns, error strings, unknown-command
suggestions, pflag's argument forms and cobra's ``stripFlags``/``Find``."""

import re

import pytest

import logparse

from move2kube_amd.cli import cobra
from move2kube_amd.cli import main as cli
from move2kube_amd.utils import log

ROOT_HELP = """\
move2kube is a tool to help optimally translate from platforms such as docker-swarm, CF to Kubernetes.

Usage:
  move2kube [command]

Available Commands:
  collect     Collect and process metadata from multiple sources.
  help        Help about any command
  plan        Plan out a move
  translate   Translate using move2kube plan
  version     Print the client version information

Flags:
  -h, --help      help for move2kube
  -v, --verbose   Enable verbose output

Use "move2kube [command] --help" for more information about a command.
"""

TRANSLATE_USAGE = """\
Usage:
  move2kube translate [flags]

Flags:
  -c, --curate            Specify whether to curate the plan with a q/a.
  -h, --help              help for translate
      --ignoreenv         Ignore data from local machine.
  -n, --name string       Specify the project name. (default "myproject")
  -o, --outpath string    Path for output. Default will be directory with the project name. (default ".")
  -p, --plan string       Specify a plan file to execute. (default "m2k.plan")
  -q, --qacache strings   Specify qa cache file locations
  -s, --source string     Specify source directory to translate. If you already have a m2k.plan then this will \
override the rootdir value specified in that plan.

Global Flags:
  -v, --verbose   Enable verbose output
"""


def _parse(argv):
    res = cobra.execute(cli.build_command_tree(), argv)
    assert not isinstance(res, int), res
    cmd, positional = res
    return cmd, positional


def test_root_help_without_a_command(capsys):
    assert cli.main([]) == 0
    assert capsys.readouterr().out == ROOT_HELP
    assert cli.main(["--help"]) == 0
    assert capsys.readouterr().out == ROOT_HELP


@pytest.mark.parametrize("argv", [["translate", "--help"], ["translate", "-h"], ["help", "translate"],
                                  ["-v", "translate", "-h"], ["translate", "-s", "x", "--help"]])
def test_translate_help(capsys, argv):
    assert cli.main(argv) == 0
    assert capsys.readouterr().out == "Translate artifacts using move2kube plan\n\n" + TRANSLATE_USAGE


def test_hidden_flags_parse_but_are_not_listed():
    cmd, _ = _parse(["translate", "--qaskip", "--qadisablecli", "--qaport", "0x1F"])
    assert cmd.value("qaskip") and cmd.value("qadisablecli") and cmd.value("qaport") == 31
    assert "qaskip" not in cmd.usage_string()


def test_unknown_command_suggestions(capsys):
    assert cli.main(["tranlate"]) == 1
    err = capsys.readouterr().err
    assert err.startswith('Error: unknown command "tranlate" for "move2kube"\n\nDid you mean this?\n\ttranslate\n\n'
                          "Run 'move2kube --help' for usage.\n")
    assert cli.main(["pl"]) == 1  # prefix match
    assert "Did you mean this?\n\tplan\n" in capsys.readouterr().err
    assert cli.main(["zzzzzz"]) == 1
    assert "Did you mean" not in capsys.readouterr().err


@pytest.mark.parametrize("argv,msg", [
    (["translate", "--bogus"], "unknown flag: --bogus"),
    (["translate", "-x"], "unknown shorthand flag: 'x' in -x"),
    (["translate", "-cx"], "unknown shorthand flag: 'x' in -x"),
    (["translate", "-s"], "flag needs an argument: 's' in -s"),
    (["translate", "--source"], "flag needs an argument: --source"),
    (["translate", "--qaport", "12a"], 'invalid argument "12a" for "--qaport" flag: strconv.ParseInt: parsing "12a": '
                                        "invalid syntax"),
    (["translate", "--qaport", "1__0"], 'invalid argument "1__0" for "--qaport" flag: strconv.ParseInt: parsing '
                                         '"1__0": invalid syntax'),
    (["translate", "-c=maybe"], 'invalid argument "maybe" for "-c, --curate" flag: strconv.ParseBool: parsing '
                                '"maybe": invalid syntax'),
    (["translate", "---x"], "bad flag syntax: ---x"),
    (["translate", "-q", 'a"b'], 'invalid argument "a\\"b" for "-q, --qacache" flag: parse error on line 1, '
                                 'column 2: bare " in non-quoted-field'),
    (["plan"], 'required flag(s) "source" not set'),
])
def test_flag_errors_print_error_and_usage(capsys, argv, msg):
    assert cli.main(argv) == 1
    err = capsys.readouterr().err
    assert err.startswith("Error: %s\nUsage:\n  move2kube %s [flags]\n" % (msg, argv[0]))
    # main.go: log.Fatalf("Error: %q", err)
    assert logparse.messages(err)[-1] == ("fatal", "Error: " + log.go_quote(msg))


def test_value_forms_and_interspersed_arguments():
    cmd, pos = _parse(["translate", "extra", "-sdir1", "-n=proj", "--outpath", "out", "-cv", "--ignoreenv=false",
                       "more", "--", "-p", "x"])
    assert cmd.value("source") == "dir1" and cmd.value("name") == "proj" and cmd.value("outpath") == "out"
    assert cmd.value("curate") is True and cmd.value("verbose") is True and cmd.value("ignoreenv") is False
    assert cmd.changed("ignoreenv") and not cmd.changed("plan") and cmd.value("plan") == "m2k.plan"
    assert pos == ["extra", "more", "-p", "x"]


def test_string_slice_is_csv_and_appends():
    cmd, _ = _parse(["translate", "-q", 'a,"b,c"', "--qacache=d", "-q", '"e""f",'])
    assert cmd.value("qacache") == ["a", "b,c", "d", 'e"f', ""]
    cmd, _ = _parse(["translate", "-q", ""])
    assert cmd.value("qacache") == [] and cmd.changed("qacache")


def test_persistent_flag_before_the_command_and_find_skips_flag_values():
    cmd, _ = _parse(["-v", "plan", "-s", "src"])
    assert cmd.name == "plan" and cmd.value("verbose")
    # cobra's stripFlags takes the word after a non-boolean flag as its value
    cmd, _ = _parse(["translate", "-n", "plan"])
    assert cmd.name == "translate" and cmd.value("name") == "plan"


def test_unknown_root_flag(capsys):
    assert cli.main(["--bogus"]) == 1
    err = capsys.readouterr().err
    assert err.startswith("Error: unknown flag: --bogus\nUsage:\n  move2kube [command]\n")


def test_help_topics(capsys):
    assert cli.main(["help"]) == 0
    assert capsys.readouterr().out == ROOT_HELP
    assert cli.main(["help", "nope"]) == 0
    err = capsys.readouterr().err
    assert err.startswith("Unknown help topic [`nope`]\nUsage:\n  move2kube [command]\n")


@pytest.mark.parametrize("text,want", [("0", 0), ("-12", -12), ("+7", 7), ("0x1f", 31), ("0o17", 15), ("017", 15),
                                       ("0b101", 5), ("1_000", 1000), ("0x_1f", 31), ("9223372036854775807",
                                                                                    (1 << 63) - 1)])
def test_parse_int_like_strconv(text, want):
    assert cobra._parse_int(text) == want


@pytest.mark.parametrize("text", ["", "-", "1_", "_1", "08", "0x", "1e3", " 1", "9223372036854775808"])
def test_parse_int_rejects_like_strconv(text):
    with pytest.raises(ValueError):
        cobra._parse_int(text)
