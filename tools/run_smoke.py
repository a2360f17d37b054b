"""Run __graft_entry__.smoke() (the driver's round-end smoke check) as a script."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__.smoke()
