"""C1 through the reference's entry line (timing probe): BPR on the bundled ml-100k."""
import sys
import time

from recbole.quick_start import run_recbole

t0 = time.time()
r = run_recbole(model='BPR', dataset='ml-100k', config_dict={
    'epochs': int(sys.argv[1]) if len(sys.argv) > 1 else 2, 'data_path': 'dataset',
    'checkpoint_dir': 'gpurun_out/saved', 'show_progress': False, 'state': 'INFO'})
print('RESULT', r['test_result'], f'{time.time() - t0:.1f}s', flush=True)
