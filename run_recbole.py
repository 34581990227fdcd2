"""Train and evaluate one model on one dataset through the MI355X path.

Same command line as the reference's script (run_recbole.py:16-31): `-m/--model`,
`-d/--dataset`, `--config_files` (space separated, later files win), `--alpha`
(forwarded as config['alpha']); any other `--key=value` flag is left on the command
line for `Config` to read, as the reference's Config does. Imports through the
`recbole` drop-in name, so this file is also what an unchanged reference user runs.
"""
import argparse

from recbole.quick_start import run_recbole


def _options(argv=None):
    cli = argparse.ArgumentParser(
        description='Run a RecBole model on the MI355X (recbole_amd) training path.')
    cli.add_argument('-m', '--model', default=None,
                     help='model class name (BPR, LightGCN, SASRec, DeepFM, ...)')
    cli.add_argument('-d', '--dataset', default=None,
                     help='dataset name: atomic files under data_path/<dataset>/')
    cli.add_argument('--config_files', default=None,
                     help='YAML config files, space separated; later files override earlier')
    cli.add_argument('--alpha', type=float, default=None,
                     help="extra hyper-parameter, forwarded as config['alpha']")
    opts, _unparsed = cli.parse_known_args(argv)   # --key=value flags: read by Config
    return opts


def main(argv=None):
    opts = _options(argv)
    files = opts.config_files.split() if opts.config_files else None
    overrides = {} if opts.alpha is None else {'alpha': opts.alpha}
    return run_recbole(model=opts.model, dataset=opts.dataset, config_file_list=files,
                       config_dict=overrides)


if __name__ == '__main__':
    main()
