import numpy as np, sys
a = np.load(sys.argv[1]); 
for f in sys.argv[2:]:
    b = np.load(f)
    d = [k for k in a.files if not np.array_equal(a[k], b[k])]
    print(f, "differs in", d, "iters", a['it'].sum(), b['it'].sum(),
          "pairs differing", int((np.abs(a['T']-b['T']).max(axis=(1,2))>0).sum()))
