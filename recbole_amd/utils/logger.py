"""Logger set-up (mirror of recbole/utils/logger.py:31-81): a file under
./log/<model>-<time>.log plus stderr."""
import logging
import os

from recbole_amd.utils.utils import ensure_dir, get_local_time


def init_logger(config):
    log_root = './log/'
    ensure_dir(log_root)
    logfile = os.path.join(log_root, f"{config['model']}-{get_local_time()}.log")
    level = {'INFO': logging.INFO, 'DEBUG': logging.DEBUG, 'WARNING': logging.WARNING,
             'ERROR': logging.ERROR, 'CRITICAL': logging.CRITICAL}.get(
        str(config['state'] or 'INFO').upper(), logging.INFO)
    fmt = logging.Formatter('%(asctime)-15s %(levelname)s  %(message)s', '%a %d %b %Y %H:%M:%S')
    fh = logging.FileHandler(logfile)
    fh.setLevel(level)
    fh.setFormatter(fmt)
    sh = logging.StreamHandler()
    sh.setLevel(level)
    sh.setFormatter(logging.Formatter('%(asctime)-15s %(levelname)s  %(message)s', '%d %b %H:%M'))
    root = logging.getLogger()
    root.handlers = []
    root.setLevel(level)
    root.addHandler(fh)
    root.addHandler(sh)
