"""Log-directory naming (reference utils/logging.py:13-51)."""
import datetime
import os

from imaginaire_amd.utils.distributed import master_only
from imaginaire_amd.utils.distributed import master_only_print as print
from imaginaire_amd.utils.meters import set_summary_writer


def get_date_uid():
    return str(datetime.datetime.now().strftime("%Y_%m%d_%H%M_%S"))


def init_logging(config_path, logdir):
    config_file = os.path.basename(config_path)
    date_uid = get_date_uid()
    log_file = '_'.join([date_uid, os.path.splitext(config_file)[0]])
    if logdir is None:
        logdir = os.path.join('logs', log_file)
    return date_uid, logdir


@master_only
def make_logging_dir(logdir):
    print('Make folder {}'.format(logdir))
    os.makedirs(logdir, exist_ok=True)
    tensorboard_dir = os.path.join(logdir, 'tensorboard')
    os.makedirs(tensorboard_dir, exist_ok=True)
    set_summary_writer(tensorboard_dir)
