require("http").createServer((q, r) => r.end("hi\n")).listen(3000);
