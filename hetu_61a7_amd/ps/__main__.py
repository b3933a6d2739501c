"""``python -m hetu_61a7_amd.ps``: run the PS role named by DMLC_ROLE (server /
scheduler) until every worker has finalised (or the launching process died)."""
import os

from .server import run_server, scheduler_init, scheduler_finish

if os.environ.get('DMLC_ROLE', 'server') == 'server':
    run_server()
else:
    scheduler_init()
    scheduler_finish()
