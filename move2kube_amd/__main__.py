import gc

from . import _cli_exit, _cli_process

_cli_process()
from .cli.main import main  # noqa: E402

gc.freeze()
_cli_exit(main())
