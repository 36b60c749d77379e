"""GPU probe: torch's current stream handle vs an ExternalStream wrapping it."""
import torch
s = torch.cuda.current_stream()
print("current", s.cuda_stream, s.stream_id)
e = torch.cuda.ExternalStream(s.cuda_stream)
print("external", e.cuda_stream, e.stream_id, e == s)
with torch.cuda.stream(e):
    c = torch.cuda.current_stream()
    print("inside", c.cuda_stream, c.stream_id, c == s)
