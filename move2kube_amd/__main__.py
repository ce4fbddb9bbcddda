import gc
import sys

from . import _cli_process

_cli_process()
from .cli.main import main  # noqa: E402

gc.freeze()
gc.enable()
sys.exit(main())
