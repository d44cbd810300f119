// TensorBoards web app frontend: list (polled), create from a PVC path (pvc://<claim>/<path>) or an
// object-store URL, delete, connect at /tensorboard/<ns>/<name>/.
(function () {
  "use strict";
  const $ = (id) => document.getElementById(id);
  let poller = null;
  async function namespaces() {
    let list = [];
    try { list = (await kf.call("GET", "/api/namespaces")).namespaces; } catch (e) { list = kf.namespace() ? [kf.namespace()] : []; }
    $("ns").innerHTML = list.map((n) => `<option>${n}</option>`).join("");
    if (!kf.namespace() && list.length) kf.setNamespace(list[0]);
    $("ns").value = kf.namespace();
    $("ns").onchange = () => kf.setNamespace($("ns").value);
  }
  async function refresh() {
    const ns = kf.namespace();
    if (!ns) return null;
    const { tensorboards } = await kf.call("GET", `/api/namespaces/${ns}/tensorboards`);
    $("rows").querySelector("tbody").replaceChildren(...tensorboards.map((tb) => {
      const tr = kf.h("tr", {});
      tr.innerHTML = `<td>${kf.statusCell(tb.status)}</td><td>${kf.esc(tb.name)}</td><td>${kf.esc(tb.logspath)}</td><td>${kf.esc(tb.age)}</td>`;
      const connect = kf.h("button", { onclick: () => window.open(`/tensorboard/${ns}/${tb.name}/`) }, "Connect");
      connect.disabled = tb.status.phase !== "ready";
      tr.append(kf.h("td", {}, connect, kf.h("button", { onclick: async () => {
        if (!confirm(`Delete TensorBoard ${tb.name}?`)) return;
        try { await kf.call("DELETE", `/api/namespaces/${ns}/tensorboards/${tb.name}`); } catch (e) { $("error").textContent = e.message; }
        poller.reset();
      } }, "Delete")));
      return tr;
    }));
    return tensorboards.map((t) => [t.name, t.status.phase]);
  }
  async function open() {
    const ns = kf.namespace();
    const [{ pvcs }, { poddefaults }] = await Promise.all([kf.call("GET", `/api/namespaces/${ns}/pvcs`),
      kf.call("GET", `/api/namespaces/${ns}/poddefaults`)]);
    $("f-pvc").innerHTML = pvcs.map((p) => `<option>${kf.esc(p)}</option>`).join("");
    $("f-configs").innerHTML = poddefaults.map((pd) => `<label class="muted"><input type="checkbox" value="${kf.esc(pd.label)}"> ${kf.esc(pd.desc)}</label><br>`).join("");
    $("dlg").showModal();
  }
  async function submit(ev) {
    if (ev.submitter && ev.submitter.value !== "ok") return;
    ev.preventDefault();
    const ns = kf.namespace(), path = $("f-path").value.trim();
    const logspath = $("f-kind").value === "pvc" ? `pvc://${$("f-pvc").value}/${path.replace(/^\//, "")}` : path;
    const configurations = [...$("f-configs").querySelectorAll("input:checked")].map((i) => i.value);
    try { await kf.call("POST", `/api/namespaces/${ns}/tensorboards`, { name: $("f-name").value, logspath, configurations }); $("dlg").close(); poller.reset(); }
    catch (e) { $("f-error").textContent = e.message; }
  }
  (async function main() {
    await namespaces();
    $("new").onclick = open;
    $("form").addEventListener("submit", submit);
    poller = new kf.Poller(refresh);
    kf.onNamespace((ns) => { $("ns").value = ns; poller.reset(); });
    poller.start();
  })();
})();
