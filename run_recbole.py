"""Command-line entry point: the reference's run_recbole.py interface
(run_recbole.py:13-31 — --model / --dataset / --config_files / --alpha ->
config_dict), through the `recbole` drop-in name."""
import argparse

from recbole.quick_start import run_recbole

if __name__ == '__main__':
    parser = argparse.ArgumentParser()
    parser.add_argument('--model', '-m', type=str, default=None, help='name of models')
    parser.add_argument('--dataset', '-d', type=str, default=None, help='name of datasets')
    parser.add_argument('--config_files', type=str, default=None, help='config files')
    parser.add_argument('--alpha', type=float, default=None, help='alpha for jsr')
    args, _ = parser.parse_known_args()
    config_file_list = args.config_files.strip().split(' ') if args.config_files else None
    config_dict = {}
    if args.alpha is not None:
        config_dict['alpha'] = args.alpha
    run_recbole(model=args.model, dataset=args.dataset, config_file_list=config_file_list,
                config_dict=config_dict)
