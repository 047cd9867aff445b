"""CPU experiment (oracle arithmetic): which bf16 rounding site of the BERT-base forward drives the
text-latent error of the HIP path.  Each site is rounded alone and all-but-one; prints max |dlatent|."""
import sys, math, torch, torch.nn.functional as F
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from oracle import ctclip_oracle as O, weights as W
torch.set_num_threads(8)
cfg = O.BASE
sd = {k:v for k,v in W.make_state_dict(cfg).items() if k.startswith('text_transformer.') or k.startswith('to_text')}
ids, mask = W.make_text(2, 128, cfg.bert.vocab_size)
def r(t): return t.bfloat16().float()
def bert(sites):
    p='text_transformer.'; b,L=ids.shape; pos=torch.arange(L)
    x = sd[p+'embeddings.word_embeddings.weight'][ids]+sd[p+'embeddings.token_type_embeddings.weight'][0]+sd[p+'embeddings.position_embeddings.weight'][pos]
    x = O._ln(x, sd[p+'embeddings.LayerNorm.weight'], sd[p+'embeddings.LayerNorm.bias'], 1e-12)
    nh, hd = 12, 64
    add_mask = (1.0-mask.float())[:,None,None,:]*torch.finfo(torch.float32).min
    R = lambda t, s: r(t) if s in sites else t
    for i in range(12):
        lp=f'{p}encoder.layer.{i}.'
        def lin(t,name): return F.linear(t, R(sd[lp+name+'.weight'],'w'), sd[lp+name+'.bias'])
        xi = R(x,'x')
        q = R(lin(xi,'attention.self.query'),'qkv').reshape(b,L,nh,hd).transpose(1,2)
        k = R(lin(xi,'attention.self.key'),'qkv').reshape(b,L,nh,hd).transpose(1,2)
        v = R(lin(xi,'attention.self.value'),'qkv').reshape(b,L,nh,hd).transpose(1,2)
        s = (q@k.transpose(-1,-2))/8 + add_mask
        a = R(s.softmax(-1),'p') @ v
        a = R(a.transpose(1,2).reshape(b,L,768),'ctx')
        x = O._ln(lin(a,'attention.output.dense')+x, sd[lp+'attention.output.LayerNorm.weight'], sd[lp+'attention.output.LayerNorm.bias'],1e-12)
        hm = R(F.gelu(lin(R(x,'x1'),'intermediate.dense')),'h')
        x = O._ln(lin(hm,'output.dense')+x, sd[lp+'output.LayerNorm.weight'], sd[lp+'output.LayerNorm.bias'],1e-12)
    t = F.linear(x[:,0], sd['to_text_latent.weight'])
    return F.normalize(t,dim=-1)
ref = bert(set())
allsites = ['w','x','qkv','p','ctx','x1','h']
print('all', (bert(set(allsites))-ref).abs().max().item())
for s in allsites:
    print(s, (bert({s})-ref).abs().max().item(), 'all-but', (bert(set(allsites)-{s})-ref).abs().max().item())
