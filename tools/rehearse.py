"""Dev tool (GPU box): run tests/mrank_body.py under torchrun exactly as
test_multirank_rehearsal_gpu does (captured pipes), printing the children's
output even when they time out.  python tools/rehearse.py [timeout_s]"""
import os
import socket
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
s = socket.socket()
s.bind(('127.0.0.1', 0))
port = s.getsockname()[1]
s.close()
env = dict(os.environ, SPARTAN_DIST_BACKEND='gloo', REHEARSAL_WORKERS='3')
cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=2',
       '--master-addr=127.0.0.1', '--master-port=%d' % port, os.path.join(ROOT, 'tests', 'mrank_body.py')]
try:
  r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=float(sys.argv[1]) if len(sys.argv) > 1 else 100)
  print('rc', r.returncode)
  print(r.stdout[-3000:])
  print(r.stderr[-6000:])
except subprocess.TimeoutExpired as e:
  print('TIMEOUT')
  print((e.stdout or b'')[-3000:] if isinstance(e.stdout, bytes) else (e.stdout or '')[-3000:])
  print((e.stderr or b'')[-8000:] if isinstance(e.stderr, bytes) else (e.stderr or '')[-8000:])
